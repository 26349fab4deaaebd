# r04 n: the deferred accounting's phases (diagnostic build)
R=$(pwd)
O=$R/gpurun_out/r04n; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/r04/sdef_phases.py > $O/sdef_phases.log 2>&1
echo "rc=$?" >> $O/rc.log
exit 0
