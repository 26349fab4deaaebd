#!/bin/bash
# Round 3 session u: k2_pa finishes its node-table claims late (the count atomics overlap the reductions).
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -3 $O/$name.log | cut -c1-900
  if [ $rc -ne 0 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
step parity 600 $PYT tests/test_gpu_wide.py tests/test_gpu_p2p.py tests/test_gpu_icmp.py tests/test_gpu_mixed.py tests/test_gpu_hubs.py tests/test_gpu_dumbbell.py tests/test_gpu_trace.py tests/test_gpu_p2p_dist.py -k "not million"
L=ns-3-dev-dnemu_amd/lib
step variants 300 python scripts/variants.py $L/libnsgpu.so $L/libnsgpu.so
step blocks 300 python scripts/p2p_blocks.py 128
step part 300 python bench.py --partitioned --no-cpu-baseline --no-secondary --steps 3
exit 0
