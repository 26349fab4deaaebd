#!/bin/bash
# GPU-box A/B runner for build variants (lib/libnsgpu_var<X>.so): one partitioned-grid bench line and the eager
# rocprofv3 kernel stats per variant, each step under its own time limit; the first failure ends the script.
# usage: bash scripts/var_bench.sh OUT VARIANT... [-- BENCH ARGS (commas for spaces)]
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
ARGS="--partitioned --no-cpu-baseline"
VARS=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then ARGS="${2//,/ }"; break; fi
  VARS+=("$1"); shift
done
mkdir -p $O
for v in "${VARS[@]}"; do
  L=$R/ns-3-dev-dnemu_amd/lib/libnsgpu_var$v.so
  [ "$v" = base ] && L=$R/ns-3-dev-dnemu_amd/lib/libnsgpu.so
  echo "[$(date +%T)] $v" >> $O/steps.log
  NSGPU_LIB=$L timeout -k 10 200 python $R/bench.py $ARGS > $O/bench_$v.log 2>&1 || { echo "$v bench FAILED" >> $O/steps.log; exit 1; }
  cd /tmp
  NSGPU_LIB=$L NSGPU_P2P_EAGER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- python3 $R/bench.py $ARGS --steps 1 --warmup 0 > $O/prof_$v.log 2>&1 || { echo "$v rocprof FAILED" >> $O/steps.log; exit 1; }
  cd $R
done
echo "[$(date +%T)] done" >> $O/steps.log
