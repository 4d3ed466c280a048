#!/bin/bash
# gpurun with retries while the pod has no free GPU slot (exit 3: nothing ran, nothing charged).  Any other exit code
# -- success, failure, refusal -- ends it.  usage: tools/gpurun_retry.sh <log> <timeout> <command>
log=$1; to=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$@" > "$log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 150
done
echo EXIT $rc >> "$log"
