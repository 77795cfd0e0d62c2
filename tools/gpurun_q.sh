#!/bin/bash
# Submit one gpurun call; while the pool reports no free box / slot (exit 3: nothing ran,
# nothing charged), wait and submit the same call again.  Any other outcome ends it.
#   bash tools/gpurun_q.sh LOG TIMEOUT CMD...
LOG=$1; TO=$2; shift 2
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "EXIT $rc" >> "$LOG"
