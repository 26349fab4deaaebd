#!/bin/bash
# Round 3, session f (re-entry): the default bench line at HEAD (wide windows on config 4, with its
# secondary entries), the in-kernel phase times, and the whole -m gpu suite.
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
step() {  # step <name> <timeout s> <command...>
  local name=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a $O/steps.log
  tail -4 $O/$name.log | cut -c1-700
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -v --timeout 300 --timeout-method thread"
step bench 500 python bench.py
step phases_wide 300 python scripts/p2p_phases.py 128
step suite 900 $PYT -m gpu tests
exit 0
