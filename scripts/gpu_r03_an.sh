#!/bin/bash
# Round 3 session an: config 5 (1M-node dumbbell) under rocprofv3 — kernel stats (eager launches: graph
# replays crash the tracer) and the FETCH / WRITE passes for profiles/traffic_dumbbell.json.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03an
mkdir -p $O
cd /tmp
export NSGPU_P2P_EAGER=1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1
echo "kt ok"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1
echo "fetch ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1
echo "write ok"
python3 $R/scripts/pmc_traffic.py $O/fetch $O/write $O/traffic_dumbbell.json k2_handle k2_pa k2_scan > $O/traffic.log 2>&1
echo "traffic ok"
