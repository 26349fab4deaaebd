#!/bin/bash
# A/B of a runtime environment setting on the default bench line (config 4, no secondaries, no CPU baseline),
# interleaved on one box: bash scripts/env_ab.sh OUT "VAR=value [VAR2=value]" [reps] [bench args...]
# Each run under its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
ENVS=$2
REPS=${3:-2}
shift 3 || shift $#
mkdir -p $O
cd $R
for r in $(seq 1 $REPS); do
  timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline "$@" > $O/a_$r.json 2> $O/a_$r.err
  timeout -k 10 200 env $ENVS python bench.py --no-secondary --no-cpu-baseline "$@" > $O/b_$r.json 2> $O/b_$r.err
done
python - "$O" "$REPS" <<'EOF'
import json, sys
o, reps = sys.argv[1], int(sys.argv[2])
for tag in "ab":
    for r in range(1, reps + 1):
        d = json.loads(open(f"{o}/{tag}_{r}.json").read().strip().splitlines()[-1])
        rl = d["roofline"]
        print(tag, r, round(d["value"] / 1e6, 2), "M ev/s", round(d["ms_per_step"], 2), "ms",
              rl.get("pipeline_ms_per_window"))
EOF
