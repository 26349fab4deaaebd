#!/bin/bash
# A/B of library builds on the default bench line (config 4, no secondaries, no CPU baseline), interleaved on one
# box: bash scripts/lib_ab.sh OUT REPS LIB_A LIB_B [LIB_C ...] (paths relative to the repo); each run under its own
# time limit, the first failure ends the script.  Extra bench arguments: BENCH_ARGS in the environment.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
REPS=$2
shift 2
mkdir -p $O
cd $R
for r in $(seq 1 $REPS); do
  i=0
  for L in "$@"; do
    NSGPU_LIB=$R/$L timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline $BENCH_ARGS > $O/v${i}_$r.json 2> $O/v${i}_$r.err
    i=$((i + 1))
  done
done
python - "$O" "$REPS" "$@" <<'PY'
import json, sys
o, reps, libs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for i, lib in enumerate(libs):
    for r in range(1, reps + 1):
        d = json.loads(open(f"{o}/v{i}_{r}.json").read().strip().splitlines()[-1])
        print(lib, r, round(d["value"] / 1e6, 2), "M ev/s", round(d["ms_per_step"], 2), "ms",
              d["roofline"].get("pipeline_ms_per_window"), flush=True)
PY
