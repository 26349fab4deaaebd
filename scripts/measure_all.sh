#!/bin/bash
# Bench lines of every workload, rocprofv3 kernel stats of the default bench (config 4, eager launches:
# the tracer cannot follow graph replays) and of the closed-loop Wi-Fi line, and the config-4 HBM traffic
# passes (FETCH_SIZE / WRITE_SIZE in separate runs) -> gpurun_out/measure.  Every GPU step has its own
# time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/measure
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_p2p_grid.log 2>&1
timeout -k 10 300 python bench.py --workload dumbbell --partitioned > $O/bench_dumbbell_partitioned.log 2>&1
timeout -k 10 300 python bench.py --partitioned --no-cpu-baseline > $O/bench_p2p_grid_partitioned.log 2>&1
timeout -k 10 300 python bench.py --workload wifi-loop > $O/bench_wifi_loop.log 2>&1
timeout -k 10 300 python bench.py --workload churn > $O/bench_churn.log 2>&1
cd /tmp
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/rocprof_p2p.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_wifil -o run --output-format csv -- python3 $R/bench.py --workload wifi-loop --steps 1 --warmup 0 --no-cpu-baseline > $O/rocprof_wifil.log 2>&1
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_grid -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $O/pmc_fetch_grid.log 2>&1
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_grid -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $O/pmc_write_grid.log 2>&1
cd $R
python scripts/pmc_traffic.py $O/pmc_fetch_grid $O/pmc_write_grid $O/traffic_p2p-grid.json k2_pa k2_handle k2_rank > $O/traffic_grid.log 2>&1
