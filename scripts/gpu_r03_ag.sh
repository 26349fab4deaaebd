#!/bin/bash
# Round 3 session ag: partitioned Wi-Fi receive subset (loopback groups, RCCL one rank) and the single
# engine's wifi parity after the receiver-range change.
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wifi_dist.py tests/test_gpu_wifi.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 5 $O/parity.log
