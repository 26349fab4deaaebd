#!/bin/bash
# Round 3 session i: k2_rank with 64-column unrolled tiles — wide parity tests, probe, bench; TLB probe.
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -12 $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step wide 400 $PYT tests/test_gpu_wide.py tests/test_gpu_p2p.py
step rank_probe 300 python scripts/rank_probe.py
step bench 300 python bench.py --no-secondary --no-cpu-baseline --steps 5
step phases 300 python scripts/p2p_phases.py 128
step tlb 120 ./scripts/probe_tlb
exit 0
