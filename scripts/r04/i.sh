# r04 i: parity (closed-loop wave-per-phy step, multi-block deferred accounting, mixed tests), the default
# bench line, variants, and rocprofv3 kernel stats (config 4 eager; the closed loop)
R=$(pwd)
O=$R/gpurun_out/r04i; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {  # name, timeout, command...: a test failure (rc 1) continues, anything else stops the script
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step wifi 400 python -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wifi_loop.py tests/test_gpu_wifi_trace.py
step p2p 500 python -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_mixed.py
step bench_default 500 python bench.py
step bench_nodefer 300 env NSGPU_P2P_NODEFER=1 python bench.py --no-cpu-baseline --no-secondary
step bench_sdefk 300 env NSGPU_P2P_SDEF_KERNEL=1 python bench.py --no-cpu-baseline --no-secondary
step bench_wifil_lane 300 env NSGPU_WIFIL_LANE=1 python bench.py --workload wifi-loop --no-cpu-baseline
step bench_dumbbell_part 300 python bench.py --workload dumbbell --partitioned --steps 2 --warmup 1
cd /tmp
step rocprof_p2p 240 env NSGPU_P2P_EAGER=1 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step rocprof_wifil 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_wifil -o run --output-format csv -- python3 $R/bench.py --workload wifi-loop --steps 1 --warmup 0 --no-cpu-baseline
step rocprof_dumbbell_part 240 env NSGPU_P2P_EAGER=1 rocprofv3 --kernel-trace --stats -d $O/rocprof_dumbbell_part -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --partitioned --steps 1 --warmup 0 --no-cpu-baseline
exit 0
