#!/bin/bash
# Round 3 session ai: rocprofv3 kernel stats + FETCH/WRITE passes of the wifi-grid run with sorted rows,
# and kernel stats of the closed-loop 10,000-phy run (deferred chunk products).
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03ai
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt_wifi -o run --output-format csv -- python3 $R/scripts/wifi_once.py 2.0 > $O/kt_wifi.log 2>&1
echo "kt_wifi ok"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_wifi -o run --output-format csv -- python3 $R/scripts/wifi_once.py 2.0 > $O/fetch_wifi.log 2>&1
echo "fetch ok"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_wifi -o run --output-format csv -- python3 $R/scripts/wifi_once.py 2.0 > $O/write_wifi.log 2>&1
echo "write ok"
python3 $R/scripts/pmc_traffic.py $O/fetch_wifi $O/write_wifi $O/traffic_wifi-grid.json k_wifi_phy k_wifi_rx_sort k_wifi_rx > $O/traffic.log 2>&1
echo "traffic ok"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_wifil -o run --output-format csv -- python3 $R/scripts/wifi_loop_scale.py 100 1.0 0.2 0 > $O/kt_wifil.log 2>&1
echo "kt_wifil ok"
