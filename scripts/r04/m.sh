# r04 m: parity and the bench line with the single-buffered stage (the accounting loads its records with the flag)
# and rocprofv3 kernel stats of config 4 (eager) and the closed loop
R=$(pwd)
O=$R/gpurun_out/r04m; mkdir -p $O
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
cd /tmp
step rocprof_p2p 240 env NSGPU_P2P_EAGER=1 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary
step rocprof_wifil 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_wifil -o run --output-format csv -- python3 $R/bench.py --workload wifi-loop --steps 1 --warmup 0 --no-cpu-baseline
exit 0
