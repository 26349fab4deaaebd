#!/bin/bash
# p2p GPU tests, then the p2p-grid HBM traffic passes (FETCH_SIZE / WRITE_SIZE, eager launches) and
# the bench line that reads them.  Every GPU step has its own time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_trace.py tests/test_gpu_icmp.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > $O/pytest_p2p.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_grid -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_fetch_grid.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_grid -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_write_grid.log 2>&1 && \
python scripts/pmc_traffic.py $O/pmc_fetch_grid $O/pmc_write_grid $O/traffic_p2p-grid.json k2_handle k2_pa k2_scan \
    > $O/traffic_grid.log 2>&1 && cp $O/traffic_p2p-grid.json profiles/ && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > $O/bench_grid.log 2>&1
rc=$?
tail -2 $O/pytest_p2p.log; cut -c1-600 $O/traffic_grid.log; tail -1 $O/bench_grid.log | cut -c1-200
exit $rc
