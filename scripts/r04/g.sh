# r04 g: (1) the drained-engine send test, eager with per-window run-control trace; (2) the closed-loop
# Wi-Fi tests with the fused epoch tail; (3) the p2p parity set and the benches
O=gpurun_out/r04g; mkdir -p $O
step() {  # name, timeout, command...: a test failure (rc 1) continues, anything else stops the script
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
export PYTHONUNBUFFERED=1
step trace 120 env NSGPU_P2P_EAGER=1 NSGPU_P2P_DEBUG=1 NSGPU_P2P_DEBUG_TRACE=1 python -m pytest -x -v -s --timeout 30 --timeout-method thread -m gpu "tests/test_gpu_mixed.py::test_send_after_engine_finished_is_refused"
step wifiloop 400 python -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wifi_loop.py tests/test_gpu_wifi_trace.py
step p2p 500 python -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_mixed.py --deselect "tests/test_gpu_mixed.py::test_send_after_engine_finished_is_refused"
step bench_default 300 python bench.py
step bench_nodefer 300 env NSGPU_P2P_NODEFER=1 python bench.py --no-cpu-baseline --no-secondary
step bench_dumbbell_part 300 python bench.py --workload dumbbell --partitioned
step bench_wifiloop 300 python bench.py --workload wifi-loop --no-cpu-baseline
exit 0
