#!/bin/bash
# tools/gpuq.sh (CPU host side) <log> <cmd>: run one gpurun call, re-queueing only while no
# box/slot is free (exit 3: nothing ran, nothing charged), after the wait gpurun asks for.
# Any other exit ends it.
LOG=$1; shift
for i in $(seq 1 40); do
  timeout 2400 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" >> $LOG 2>&1
  rc=$?
  echo "EXIT $rc (attempt $i)" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  w=$(tail -5 $LOG | grep -o "retry in [0-9]*s" | tail -1 | grep -o "[0-9]*")
  sleep $(( ${w:-120} + 15 ))
done
