#!/bin/bash
# Round 3 session aj: X1 all-gathered in place (k_dfin2's last reader resets the header) — the partitioned
# p2p tests, then the partitioned window on one rank.
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_p2p_dist.py tests/test_gpu_hubs.py tests/test_gpu_icmp.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --partitioned --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_part.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -n 1 $O/bench_part.log | cut -c1-400
