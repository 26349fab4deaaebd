# Bench lines of every workload + rocprofv3 kernel stats of the default bench (config 4) at HEAD.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/measure
mkdir -p $O
cd $R
timeout -k 10 200 python -u bench.py > $O/bench_p2p_grid.log 2>&1
timeout -k 10 200 python -u bench.py --partitioned --no-cpu-baseline > $O/bench_p2p_grid_partitioned.log 2>&1
timeout -k 10 200 python -u bench.py --workload wifi-grid > $O/bench_wifi_grid.log 2>&1
timeout -k 10 200 python -u bench.py --workload dumbbell > $O/bench_dumbbell.log 2>&1
timeout -k 10 200 python -u bench.py --workload churn > $O/bench_churn.log 2>&1
cd /tmp
# (under the tracer the window kernels are launched one by one: graph replays crash the tracer)
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/rocprof_p2p.log 2>&1
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_part -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --partitioned > $O/rocprof_part.log 2>&1
