#!/bin/bash
# Round 3, session c: wide windows (local records) — the p2p GPU tests first (they compare every run with
# the oracle), then config 4's bench line wide and narrow.  Each GPU step has its own time limit; a
# fault, abort or timeout ends the script (an ordinary test failure does not).
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -5 $O/$name.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step wide 400 $PYT tests/test_gpu_wide.py
step p2p 400 $PYT -x tests/test_gpu_p2p.py
step suite 600 $PYT -m gpu tests -k "not million"
step bench_wide 300 python bench.py --no-secondary --steps 5
step bench_narrow 300 env NSGPU_P2P_NARROW=1 python bench.py --no-secondary --steps 5 --no-cpu-baseline
exit 0
