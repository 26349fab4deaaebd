#!/bin/bash
# Diagnostic: the open-loop Wi-Fi grid (config 3) at several phys per block of k_wifi_phy_lds
# (NSGPU_WIFI_PHYS_PER_BLOCK), interleaved: bash scripts/wifi_ppb_sweep.sh OUT REPS P1 P2 ...
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
cd $R
for r in $(seq 1 $REPS); do
  for P in "$@"; do
    NSGPU_WIFI_PHYS_PER_BLOCK=$P timeout -k 10 200 python bench.py --workload wifi-grid --no-secondary --no-cpu-baseline \
      --steps 3 > $O/p${P}_$r.json 2> $O/p${P}_$r.err
  done
done
python - "$O" "$REPS" "$@" <<'PY'
import json, sys
o, reps, ps = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for p in ps:
    for r in range(1, reps + 1):
        d = json.loads(open(f"{o}/p{p}_{r}.json").read().strip().splitlines()[-1])
        rl = d["roofline"]
        print("P", p, r, round(d["value"] / 1e9, 3), "G ev/s", round(d["ms_per_step"], 2), "ms", "phy kernel",
              round(rl.get("kernel_ms", 0), 2), "ms", d.get("extra"), flush=True)
PY
