# r04 s: rocprofv3 kernel stats of the closed-loop Wi-Fi line
R=$(pwd)
O=$R/gpurun_out/r04s; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_wifil -o run --output-format csv -- python3 $R/bench.py --workload wifi-loop --steps 1 --warmup 0 --no-cpu-baseline > $O/rocprof_wifil.log 2>&1
echo "rc=$?" >> $O/rc.log
