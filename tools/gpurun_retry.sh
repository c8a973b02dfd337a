#!/bin/bash
# (client side, this container) re-submit a gpurun call only while the pool reports no free slot
# or box -- status=transient / exit 3: nothing ran, nothing was charged.  usage: tools/gpurun_retry.sh LOG gpurun-args...
LOG=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun "$@" > $LOG.tmp 2>&1
  rc=$?
  cat $LOG.tmp >> $LOG
  if grep -q "status=transient" $LOG.tmp || [ $rc = 3 ]; then sleep 90; continue; fi
  exit $rc
done
