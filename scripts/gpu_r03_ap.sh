#!/bin/bash
# Round 3 session ap (final): the whole -m gpu suite, smoke, and the default bench line (p2p-grid + secondaries).
export TMPDIR=/tmp
O=gpurun_out/r03ap
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/ > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -n 2 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -n 1 $O/bench_default.log | cut -c1-300
