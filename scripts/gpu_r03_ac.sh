#!/bin/bash
# Round 3 session ac: k_wl_step per-epoch lane times (diagnostic build).
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 300 python -u scripts/wifil_probe.py > $O/probe.log 2>&1; echo "probe rc=$?"; tail -3 $O/probe.log
