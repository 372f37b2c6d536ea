#!/bin/bash
# usage: gpuq.sh LOG TIMEOUT CMD -- retries only while no GPU slot is free (nothing charged)
LOG=$1; TO=$2; shift 2
for i in 1 2 3 4 5 6 7 8; do
  timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient\|slot(s) on this pod are busy" $LOG && [ $rc -ne 0 ]; then sleep 200; continue; fi
  break
done
echo "GPUQ_DONE rc=$rc" >> $LOG
