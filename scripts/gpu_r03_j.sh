#!/bin/bash
# Round 3 session j: k2_scan with odd rank spans (no LDS bank conflicts), k2_pa local slots to LMAX;
# parity, bench, phases and per-block times of the wide window.
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -14 $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step wide 500 $PYT tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_icmp.py tests/test_gpu_mixed.py
step bench 300 python bench.py --no-secondary --no-cpu-baseline --steps 5
step phases 300 python scripts/p2p_phases.py 128
step blocks 300 python scripts/p2p_blocks.py 128
exit 0
