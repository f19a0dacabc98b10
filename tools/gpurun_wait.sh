#!/bin/bash
# Submit one gpurun call, waiting for a box: re-submits only while gpurun answers 3 (no box or
# slot free / transient preparation failure: nothing ran, nothing charged), at most 12 times.
# Any other exit -- including a failed GPU command -- ends it.  usage: tools/gpurun_wait.sh <log> <timeout> <cmd>
log=$1; lim=$2; shift 2
for i in $(seq 1 12); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "rc=$rc" >> "$log"
exit $rc
