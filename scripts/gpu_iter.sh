set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_hubs.py tests/test_gpu_p2p.py tests/test_gpu_dumbbell.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t2.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && \
timeout -k 10 300 python scripts/dumbbell_timing.py 32767 > gpurun_out/db.log 2>&1 && \
timeout -k 10 400 python scripts/dumbbell_timing.py 499999 >> gpurun_out/db.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_db -o db -- python3 scripts/dumbbell_timing.py 131071 > gpurun_out/prof_db.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR" gpurun_out/t2.log | tail -30; cat gpurun_out/bench.log gpurun_out/db.log
exit $rc
