#!/bin/bash
# Round 3 session ae: wifi-grid sorted reception rows (k_wifi_rx_sort, MODE 2 per-phy chain) — the
# wifi parity suite, then the wifi-grid bench line (sorted) and the unsorted store for comparison.
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wifi.py > $O/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -n 3 $O/parity.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload wifi-grid --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_wifi.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -n 1 $O/bench_wifi.log | cut -c1-600
