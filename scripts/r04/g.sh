# r04 g: the drained-engine send test, eager with per-window run-control trace
O=gpurun_out/r04g; mkdir -p $O
T="tests/test_gpu_mixed.py::test_send_after_engine_finished_is_refused"
NSGPU_P2P_EAGER=1 NSGPU_P2P_DEBUG=1 NSGPU_P2P_DEBUG_TRACE=1 timeout -k 10 120 python -u -m pytest -x -v -s --timeout 30 --timeout-method thread -m gpu $T > $O/trace.log 2>&1
rc=$?; echo "rc=$rc" >> $O/rc.log
exit 0
