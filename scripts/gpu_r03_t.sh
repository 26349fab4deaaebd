#!/bin/bash
# Round 3 session t: partitioned window on one rank, A/B on one box: the committed library (q) against the
# working tree (per-rank lane reads, k_dfin2 one-trip loads), twice each.
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
L=ns-3-dev-dnemu_amd/lib
for v in q cur q cur; do
  if [ $v = q ]; then export NSGPU_LIB=$PWD/$L/libnsgpu_q.so; else unset NSGPU_LIB; fi
  timeout -k 10 200 python bench.py --partitioned --no-cpu-baseline --no-secondary --steps 3 > $O/part_$v.log 2>&1 || exit $?
  echo "$v $(grep '^{' $O/part_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],2))')" | tee -a $O/ab.log
done
exit 0
