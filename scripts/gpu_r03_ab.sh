#!/bin/bash
# Round 3 session ab: closed-loop Wi-Fi NiChanges insertion shifts 8 entries a trip;
# SendPacket, pinned state reads — parity tests, then the 10,000-phy timing.
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wifi_loop.py tests/test_gpu_plugin.py tests/test_gpu_sched.py tests/test_gpu_mixed.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 32 0.02 0.1 1 > $O/loop32.log 2>&1; echo "loop32 rc=$?"; tail -2 $O/loop32.log
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/loop100.log 2>&1; echo "loop100 rc=$?"; tail -2 $O/loop100.log
