"""Summarise a scripts/var_bench.sh run: each variant's bench value / ms and its kernels' average durations."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
for b in sorted(glob.glob(os.path.join(out, "bench_*.log"))):
    v = os.path.basename(b)[6:-4]
    line = [x for x in open(b) if x.startswith("{")]
    d = json.loads(line[-1]) if line else {}
    print(f"{v:6s} value {d.get('value', 0) / 1e6:8.2f} M  {d.get('ms_per_step', 0):8.2f} ms")
    f = os.path.join(out, f"prof_{v}", "run_kernel_stats.csv")
    if os.path.exists(f):
        for r in csv.DictReader(open(f)):
            if float(r["TotalDurationNs"]) > 2e6:
                print(f"    {r['Name'][:52]:52s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.2f} us")
