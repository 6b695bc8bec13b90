#!/bin/bash
# Submit one gpurun call, resubmitting only while the pod has no free slot (exit 3: nothing ran,
# nothing charged). Any other exit code, including a failed GPU step, ends it.
#   tools/gpurun_wait.sh TIMEOUT 'command' LOG
T=$1; CMD=$2; LOG=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  echo "rc=$rc" >> "$LOG"
  [ $rc -ne 3 ] && exit $rc
  sleep 150
done
exit 3
