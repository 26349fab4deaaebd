#!/bin/bash
# Round 3 session aq: the headline line twice and its rocprofv3 kernel stats on the same box (eager launches:
# graph replays crash the tracer), for the roofline cross-check.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03aq
mkdir -p $O
cd $R
for i in 1 2; do timeout -k 10 150 python -u bench.py --no-secondary --no-cpu-baseline > $O/b$i.log 2>&1; tail -n 1 $O/b$i.log | cut -c1-160; done
cd /tmp
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary > $O/rocprof_p2p.log 2>&1
echo "rocprof ok"
