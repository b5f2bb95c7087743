#!/bin/bash
# Run one gpurun call, waiting out "no free box / slot" answers (exit 3 or status=transient: nothing
# ran, nothing charged).  Any other outcome -- success or a failure of the command itself -- ends it:
# a GPU command that failed is never re-run from here.
# usage: scripts/gpurun_when_free.sh <log> <timeout_s> <command...>
LOG=${1:?log}; TO=${2:?timeout}; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || { [ $rc -ne 0 ] && grep -q "status=transient" "$LOG"; }; then
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
