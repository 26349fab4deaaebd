#!/bin/bash
# Round 3, first GPU session: the new plugin-path tests, the whole -m gpu suite, the host-closure
# plugin bench (scripts/sched_bench.py), the default bench line (with its `secondary` entries), and the
# 1M-node dumbbell tests.  Every GPU step has its own time limit; a step that faults, aborts or times
# out ends the script (an ordinary test failure, exit 1, does not).
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -3 $O/$name.log | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step plugin 300 $PYT tests/test_gpu_plugin.py tests/test_gpu_sched.py tests/test_gpu_mixed.py
step suite 600 $PYT -m gpu tests -k "not million"
step sched_bench 400 python scripts/sched_bench.py 5000000
step bench 500 python bench.py
step million_single 400 $PYT tests/test_gpu_dumbbell.py -k "million_nodes_single"
step million_part 400 $PYT tests/test_gpu_dumbbell.py -k "million_nodes_eight"
exit 0
