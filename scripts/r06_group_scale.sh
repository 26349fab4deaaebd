#!/bin/bash
# k_gtile (and the rest of the partitioned window) per launch at N = 1, 2, 4, 8 loopback partitions of config 4
# weak-scaled (scripts/p2p_group_scale.py), plus each N's graph-replay wall time.  Usage: scripts/r06_group_scale.sh OUT
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/${1:-gpurun_out/r06g}
mkdir -p $O
export TMPDIR=/tmp
for N in 1 2 4 8; do
  timeout -k 10 150 python3 $R/scripts/p2p_group_scale.py $N 128 2 > $O/wall_n$N.json
  cd /tmp
  NSGPU_P2P_EAGER=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_n$N -o run --output-format csv -- python3 $R/scripts/p2p_group_scale.py $N 128 1 > $O/prof_n$N.log 2>&1
  rm -f $O/prof_n$N/run_kernel_trace.csv
  cd $R
done
