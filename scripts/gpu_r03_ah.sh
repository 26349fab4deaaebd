#!/bin/bash
# Round 3 session ah: wifi-grid through the partitioned engine on one rank (RCCL with one rank) against the
# single engine.
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload wifi-grid --partitioned --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_wifi_part1.log 2>&1; rc=$?; echo "part1 rc=$rc"; tail -n 1 $O/bench_wifi_part1.log | cut -c1-300
