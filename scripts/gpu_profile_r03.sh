#!/bin/bash
# Round-3 profile set of the headline step at HEAD: rocprofv3 kernel trace of the
# 1-GPU bench, in-kernel phase stamps of the 2-launch step, the bench at the driver's
# flags and the long run.  Each GPU step has its own limit; the first failure stops it.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
step prof_mnist 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mnist -o bench -- python3 bench.py --gpus 1 --steps 500 --warmup 50
step stamps 120 python -u scripts/stamps.py 64
step bench_driver 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_driver.log | cut -c1-200
step bench_long 200 python -u bench.py --phases 50
tail -1 gpurun_out/bench_long.log | cut -c1-200
