#!/bin/bash
# Round 3 session aa: the lockstep deep-chain test, and how many exact chain compares it makes.
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py > $O/wide.log 2>&1; echo "wide rc=$?"; tail -3 $O/wide.log
timeout -k 10 200 python -u scripts/tie_probe.py > $O/ties.log 2>&1; echo "ties rc=$?"; tail -2 $O/ties.log
