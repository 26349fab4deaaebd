#!/bin/bash
# Round 3 session ao: closed-loop status block in one copy (parity + the 10,000-phy timing), the partitioned
# Wi-Fi tests after the create clean-up, then the config 5 profiling (gpu_r03_an.sh).
export TMPDIR=/tmp
O=gpurun_out/r03ao
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wifi_loop.py tests/test_gpu_plugin.py tests/test_gpu_wifi_dist.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/loop100.log 2>&1; rc=$?; echo "loop100 rc=$rc"; tail -n 2 $O/loop100.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_r03_an.sh
