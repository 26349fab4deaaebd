# r04 p: coalesced stage layout + padded LDS in the deferred accounting: p2p parity, then the bench
R=$(pwd)
O=$R/gpurun_out/r04p; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_p2p.py tests/test_gpu_wide.py tests/test_gpu_mixed.py tests/test_gpu_hubs.py tests/test_gpu_icmp.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-secondary --steps 5 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 env NSGPU_P2P_SDEF_KERNEL=1 python bench.py --no-cpu-baseline --no-secondary --steps 2 > $O/bench_sk.log 2>&1
echo "bench_sk rc=$?" >> $O/rc.log
exit 0
