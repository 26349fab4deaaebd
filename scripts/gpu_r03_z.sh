#!/bin/bash
# Round 3 session z: the wifi-loop bench workload alone, then the default bench line with its secondaries.
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload wifi-loop --steps 2 --warmup 1 > $O/loop.log 2>&1; echo "loop rc=$?"; tail -1 $O/loop.log | cut -c1-2500
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"
