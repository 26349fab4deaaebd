#!/bin/bash
# (r06 bisect of config 4's k2_handle / k2_pa times) the default bench line from worktrees of earlier commits
# (ab_<commit>/, each with its own build) interleaved with this tree: bash scripts/r06_ab_old.sh OUT REPS DIR...
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=$(pwd); O=$R/gpurun_out/$1; REPS=$2; shift 2; mkdir -p $O
for r in $(seq 1 $REPS); do
  for d in "$@"; do
    (cd $R/$d && timeout -k 10 200 python bench.py --no-secondary --no-cpu-baseline $BENCH_ARGS > $O/${d//\//_}_$r.json 2> $O/${d//\//_}_$r.err)
  done
done
