#!/bin/bash
# Round 3 session g: where k2_rank's time goes (wide windows), and the narrow engine on the same box.
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -12 $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step rank_probe 300 python scripts/rank_probe.py
NSGPU_P2P_NARROW=1 step bench_narrow 300 python bench.py --no-secondary --no-cpu-baseline --steps 5
exit 0
