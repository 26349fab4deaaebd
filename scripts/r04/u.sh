# r04 u: the whole GPU test suite, smoke() and the default bench line of the final tree
R=$(pwd)
O=$R/gpurun_out/r04u; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> $O/rc.log
exit $rc
