#!/bin/bash
# Round 3 session v: the closed-loop Wi-Fi PHY at config-3 scale (10,000 phys), timed; a 32x32 run against
# the oracle.
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 32 0.02 0.1 1 > $O/loop32.log 2>&1; echo "loop32 rc=$?"; cat $O/loop32.log | tail -3
timeout -k 10 300 python -u scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/loop100.log 2>&1; echo "loop100 rc=$?"; cat $O/loop100.log | tail -3
