# r04 final: the whole GPU test suite, then every measurement (scripts/measure_all.sh)
R=$(pwd)
O=$R/gpurun_out/r04final; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/rc.log; [ $rc -ne 0 ] && exit $rc
bash scripts/measure_all.sh
rc=$?; echo "measure rc=$rc" >> $O/rc.log
exit $rc
