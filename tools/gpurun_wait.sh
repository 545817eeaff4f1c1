#!/bin/bash
# Submit one gpurun call, re-submitting only while the pool has no box for it
# (a transient status: nothing ran, nothing charged); any other outcome ends
# the loop.  usage: tools/gpurun_wait.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "status=ok" $LOG; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-150} + 20 ))
    continue
  fi
  exit $rc
done
exit 3
