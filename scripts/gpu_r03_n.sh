#!/bin/bash
# Round 3 session n: the config-4 wide pipeline's measurement set — rocprofv3 kernel stats (eager launches),
# HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one counter a run), the traffic file the bench reads, and the
# default bench line (with its secondary entries).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03n
mkdir -p $O
cd $R
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary"
cd /tmp
NSGPU_P2P_EAGER=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $B > $O/rocprof_p2p.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $O/pmc_fetch.log 2>&1 && \
NSGPU_P2P_EAGER=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary > $O/pmc_write.log 2>&1 && \
cd $R && python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/traffic_p2p-grid.json k2_pa k2_handle k2_rank k2_scan > $O/traffic.log 2>&1 && \
cp $O/traffic_p2p-grid.json profiles/ && \
timeout -k 10 500 python -u bench.py > $O/bench.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 $O/rocprof_p2p.log | cut -c1-300; cat $O/traffic.log | cut -c1-800; tail -1 $O/bench.log | cut -c1-1500
exit $rc
