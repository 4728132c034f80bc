#!/bin/bash
# gpurun with retries (usage: scripts/gpurun_retry.sh OUTFILE <gpurun args>) while no box / slot is free (exit 3 / transient); nothing runs then
out=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out && [ $rc -ne 0 ]; then sleep 150; continue; fi
  break
done
echo "final rc=$rc" >> $out
