#!/bin/bash
# dev helper (container side): submit one gpurun call, resubmitting only while the pool has no free slot
# (exit 3: nothing ran, nothing charged).  usage: tools/gpurun_wait.sh <log> <timeout> <command>
LOG=$1; T=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 90
done
echo "gpurun rc=$rc" >> "$LOG"
