# r04 c: deferred pipeline parity (run-mode fix, accounting folded into k2_rank) + benches
set -e
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_mixed.py tests/test_gpu_wifi_trace.py > $O/pytest_p2p.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1
NSGPU_P2P_SDEF_KERNEL=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $O/bench_sdefk.log 2>&1
NSGPU_P2P_NODEFER=1 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary > $O/bench_nodefer.log 2>&1
timeout -k 10 300 python -u bench.py --workload dumbbell --partitioned > $O/bench_dumbbell_part.log 2>&1
