#!/bin/bash
# One GPU-box session: the -m gpu suite, smoke, and the bench line of every workload (with CPU baselines).
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_grid.log 2>&1 && \
timeout -k 10 300 python bench.py --workload dumbbell --steps 3 --warmup 1 > gpurun_out/bench_dumbbell.log 2>&1 && \
timeout -k 10 300 python bench.py --workload wifi-grid --steps 2 --warmup 1 > gpurun_out/bench_wifi.log 2>&1 && \
timeout -k 10 300 python bench.py --workload churn --steps 3 --warmup 1 > gpurun_out/bench_churn.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log
for f in grid dumbbell wifi churn; do tail -1 gpurun_out/bench_$f.log | cut -c1-400; done
exit $rc
