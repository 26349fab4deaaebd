set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/p2p_phases.py 128 > gpurun_out/phases.log 2>&1 && \
timeout -k 10 60 ./scripts/probe_latency > gpurun_out/latency.log 2>&1
rc=$?
cat gpurun_out/phases.log gpurun_out/latency.log
exit $rc
