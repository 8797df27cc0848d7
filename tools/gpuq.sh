#!/bin/bash
# tools/gpuq.sh (CPU host side) <log> <cmd>: run one gpurun call, re-queueing only while no box/slot is free (exit 3:
# nothing ran, nothing charged). Any other exit ends it.
LOG=$1; shift
for i in $(seq 1 30); do
  timeout 2400 /usr/local/graft/bin/gpurun --timeout 1200 -- "$@" > $LOG 2>&1
  rc=$?
  echo "EXIT $rc (attempt $i)" >> $LOG
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
