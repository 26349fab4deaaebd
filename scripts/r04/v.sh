# r04 v: rocprofv3 kernel stats of the default bench on the final tree (eager launches)
R=$(pwd)
O=$R/gpurun_out/r04v; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/rocprof_p2p.log 2>&1
echo "rc=$?" >> $O/rc.log
