#!/bin/bash
# GPU-box session for p2p engine work: the p2p parity tests, then the config-4 and config-5 bench lines
# (no CPU baseline) and per-kernel times.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_hubs.py tests/test_gpu_dumbbell.py tests/test_gpu_trace.py tests/test_gpu_mixed.py tests/test_gpu_reference_fixtures.py tests/test_gpu_p2p_dist.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_p2p.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_grid.log 2>&1 && \
timeout -k 10 200 python bench.py --workload dumbbell --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_dumbbell.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_p2p.log
for f in grid dumbbell; do python -c "
import json
d=json.loads(open('gpurun_out/bench_$f.log').read().strip().splitlines()[-1])
r=d['roofline']
print('$f', round(d['value']/1e6,2),'Mev/s', round(d['ms_per_step'],2),'ms/step', r.get('pipeline_ms_per_window'), d['config'].get('windows_per_step'))
" 2>/dev/null || tail -3 gpurun_out/bench_$f.log; done
exit $rc
