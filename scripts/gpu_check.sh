#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ROUND=${ROUND:-r01}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$ROUND -o bench \
    -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$ROUND -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$ROUND -o pmc \
    -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 && \
python scripts/pmc_traffic.py gpurun_out/pmc_fetch_$ROUND gpurun_out/pmc_write_$ROUND k_pa gpurun_out/traffic_p2p-grid.json
rc=$?
tail -5 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -1 gpurun_out/bench.log
exit $rc
