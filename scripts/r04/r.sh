# r04 r: closed-loop Wi-Fi order kernel with packed keys: its tests, then the wifi-loop bench line
R=$(pwd)
O=$R/gpurun_out/r04r; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_wifi_loop.py tests/test_gpu_wifi_trace.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload wifi-loop > $O/bench_wifi_loop.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/rc.log
exit $rc
