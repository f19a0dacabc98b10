#!/bin/bash
# Submit one gpurun call, waiting for a box: re-submits only while gpurun answers 3 (no box or
# slot free / transient preparation failure: nothing ran, nothing charged), at most 20 times, sleeping as long as gpurun asks.
# Any other exit -- including a failed GPU command -- ends it.  usage: tools/gpurun_wait.sh <log> <timeout> <cmd>
log=$1; lim=$2; shift 2
for i in $(seq 1 20); do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  w=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1); sleep $(( ${w:-60} + 15 ))
done
echo "rc=$rc" >> "$log"
exit $rc
