#!/bin/bash
# GPU-box session: the -m gpu tests named on the command line (default: all), one process, logged to
# gpurun_out/pytest_gpu.log.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
grep -E "FAIL|Error|^E |passed|failed|s$" gpurun_out/pytest_gpu.log | tail -25
exit $rc
