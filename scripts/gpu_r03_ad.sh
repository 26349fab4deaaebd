#!/bin/bash
# Round 3 session ad: closed-loop Wi-Fi chunk products deferred to k_wl_per (lane-parallel error-rate
# models) — parity, then the 10,000-phy timing and the per-lane probe.
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wifi_loop.py tests/test_gpu_plugin.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 32 0.02 0.1 1 > $O/loop32.log 2>&1; rc=$?; echo "loop32 rc=$rc"; tail -n 2 $O/loop32.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/loop100.log 2>&1; rc=$?; echo "loop100 rc=$rc"; tail -n 2 $O/loop100.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wifil_probe.py > $O/probe.log 2>&1; echo "probe rc=$?"; tail -n 3 $O/probe.log
