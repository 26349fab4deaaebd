set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace.py -k "first_cc or random_topology_trace" -x -v --timeout 120 --timeout-method thread > gpurun_out/t1.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_trace.py tests/test_gpu_hubs.py -v --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1
rc=$?
tail -3 gpurun_out/t1.log; grep -E "PASS|FAIL|ERROR" gpurun_out/t2.log | tail -40
exit $rc
