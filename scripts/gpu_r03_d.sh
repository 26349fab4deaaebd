#!/bin/bash
# Round 3, session d: wide windows with the ranking in k2_scan — divergence diagnostic
# (scripts/wide_debug.py), the wide tests, the partitioned 65,536-node dumbbell (X1 header padding), the
# 128 x 128 grid test, config 4's bench line wide and narrow, then the closed-loop Wi-Fi tests.
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -12 $O/$name.log | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step wide_debug 300 python scripts/wide_debug.py
step wide 400 $PYT tests/test_gpu_wide.py
step hubs 300 $PYT tests/test_gpu_hubs.py -k "65536_nodes_eight"
step p2p 400 $PYT tests/test_gpu_p2p.py
step bench_wide 300 python bench.py --no-secondary --steps 5
step bench_narrow 300 env NSGPU_P2P_NARROW=1 python bench.py --no-secondary --steps 5 --no-cpu-baseline
step wifi_loop 400 $PYT tests/test_gpu_wifi_loop.py
exit 0
