#!/bin/bash
# gpurun helper: run named steps, each under its own time limit, stop at the first
# fault/abort/timeout.  usage: scripts/gpu_run.sh "name:limit:cmd" ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; lim=${rest%%:*}; cmd=${rest#*:}
  echo "=== $name (limit ${lim}s): $cmd"
  timeout -k 10 "$lim" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
done
