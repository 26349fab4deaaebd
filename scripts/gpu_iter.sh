set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?
grep -E "FAIL|ERROR|^E |passed|failed" gpurun_out/t4.log | tail -30
exit $rc
