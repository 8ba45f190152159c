#!/bin/bash
# Run one gpurun command, retrying only while the pool has no box for it (nothing ran, nothing
# charged: status=transient / exit 3).  A run that started is never repeated.
# usage: tools/gpurun_when_free.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    sleep 90
    continue
  fi
  exit $rc
done
exit 3
