#!/bin/bash
# Round 3 session al: hub blocks scan the window 8 batches a memory trip — hub / dumbbell / icmp parity,
# then the dumbbell (config 5) bench line.
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_hubs.py tests/test_gpu_dumbbell.py tests/test_gpu_icmp.py tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_p2p_dist.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload dumbbell --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_dumbbell.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -n 1 $O/bench_dumbbell.log | cut -c1-300
timeout -k 10 200 python -u scripts/hub_phases.py > $O/hub_phases.log 2>&1; echo "hub rc=$?"; tail -n 6 $O/hub_phases.log
