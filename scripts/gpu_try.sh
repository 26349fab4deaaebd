#!/bin/bash
# Submits one gpurun call, re-submitting only while the pool has no free box ("transient": nothing ran,
# nothing charged).  Usage: scripts/gpu_try.sh <timeout-s> <log> <command...>
T=$1; LOG=$2; shift 2
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  if grep -q "status=transient" "$LOG"; then
    sleep 90
    continue
  fi
  break
done
tail -5 "$LOG"
