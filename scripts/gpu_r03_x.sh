#!/bin/bash
# Round 3 session x: where the closed-loop Wi-Fi run's time goes (rocprofv3 kernel trace + stats).
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03x
mkdir -p $O
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/prof.log 2>&1
echo "rc=$?"
tail -2 $O/prof.log | cut -c1-300
head -20 $O/prof/run_kernel_stats.csv 2>/dev/null || find $O/prof -name "*kernel_stats.csv" -exec head -20 {} \;
