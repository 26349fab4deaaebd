#!/bin/bash
# Round 3 session o: checkpoint at HEAD — the default bench line (config 4 wide, secondaries, CPU
# baselines, PMC traffic from profiles/), smoke(), and the whole -m gpu suite.
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -4 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step bench 500 python -u bench.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step suite 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests
exit 0
