#!/bin/bash
# Round 3 session h: k2_rank with precomputed chain words — wide-window parity tests, probe, bench.
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -12 $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step wide 400 $PYT tests/test_gpu_wide.py tests/test_gpu_p2p.py
step rank_probe 300 python scripts/rank_probe.py
step bench 300 python bench.py --no-secondary --no-cpu-baseline --steps 5
exit 0
