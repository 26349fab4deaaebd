#!/bin/bash
# End-of-round measurement session (round 2, session 3): per-kernel trace summaries and HBM traffic counters (separate
# --pmc passes) of the p2p-grid and wifi-grid workloads, then every workload's bench line (which
# reads profiles/traffic_<workload>.json written here).  Every GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02s3
mkdir -p $O
NSGPU_P2P_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_grid -o run \
    -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/trace_grid.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_grid -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch_grid.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_grid -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write_grid.log 2>&1 && \
python scripts/pmc_traffic.py $O/pmc_fetch_grid $O/pmc_write_grid profiles/traffic_p2p-grid.json k2_handle k2_pa k2_scan \
    > $O/traffic_grid.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_wifi -o run \
    -- python3 bench.py --workload wifi-grid --steps 1 --warmup 1 --no-cpu-baseline > $O/trace_wifi.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_wifi -o pmc \
    -- python3 bench.py --workload wifi-grid --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch_wifi.log 2>&1 && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_wifi -o pmc \
    -- python3 bench.py --workload wifi-grid --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write_wifi.log 2>&1 && \
python scripts/pmc_traffic.py $O/pmc_fetch_wifi $O/pmc_write_wifi profiles/traffic_wifi-grid.json k_wifi_phy \
    > $O/traffic_wifi.log 2>&1 && \
cp profiles/traffic_p2p-grid.json profiles/traffic_wifi-grid.json $O/ && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > $O/bench_grid.log 2>&1 && \
timeout -k 10 300 python bench.py --workload dumbbell --steps 3 --warmup 1 > $O/bench_dumbbell.log 2>&1 && \
timeout -k 10 300 python bench.py --workload wifi-grid --steps 2 --warmup 1 > $O/bench_wifi.log 2>&1 && \
timeout -k 10 300 python bench.py --workload churn --steps 3 --warmup 1 > $O/bench_churn.log 2>&1 && \
timeout -k 10 300 python bench.py --partitioned --steps 3 --warmup 1 > $O/bench_grid_partitioned.log 2>&1
rc=$?
cat $O/traffic_grid.log $O/traffic_wifi.log 2>/dev/null | cut -c1-300
for f in grid dumbbell wifi churn grid_partitioned; do tail -1 $O/bench_$f.log 2>/dev/null | cut -c1-300; done
exit $rc
