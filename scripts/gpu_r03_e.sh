#!/bin/bash
# Round 3, session e: sorted runs end after a cut same-ts group (k_trim), the local-record ranking in
# k2_scan with one LDS load per group member, the closed-loop Wi-Fi tests; config 4 wide bench + phases.
export TMPDIR=/tmp
O=gpurun_out/r03e5
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -8 $O/$name.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step wide 400 $PYT tests/test_gpu_wide.py
step runs 500 $PYT tests/test_gpu_hubs.py tests/test_gpu_dumbbell.py -k "not million"
step wifi_loop 400 $PYT tests/test_gpu_wifi_loop.py
step bench_wide 300 python bench.py --no-secondary --steps 5
step phases_wide 300 python scripts/p2p_phases.py 128
exit 0
