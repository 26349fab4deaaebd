# (diagnostic, r06) the closed-loop Wi-Fi epoch with another engine's stream alive (bench.py's order)
set -e
O=gpurun_out/${1:-r06f}; mkdir -p $O
P="timeout -k 10 300 python scripts/wifil_interference.py nofresh"
$P p2p_norun > $O/norun.log 2>&1
$P p2p6 close_p2p > $O/p2p6_close.log 2>&1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_nocpu.json 2>&1
