# Per-kernel averages of the partitioned engine on one rank (RCCL with one rank), kernels launched eagerly
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/part
mkdir -p $O
NSGPU_P2P_EAGER=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run \
    -- python3 bench.py --partitioned --steps 2 --warmup 1 --no-cpu-baseline > $O/trace.log 2>&1
