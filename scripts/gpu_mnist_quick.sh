#!/bin/bash
# Quick MNIST iteration: fused-engine GPU tests, phase stamps, long bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -60 "gpurun_out/$name.log"; exit $rc; fi
}
step t_fused 400 python -u -m pytest tests/test_fused_convnet_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
tail -2 gpurun_out/t_fused.log
step stamps2 120 python -u scripts/stamps.py 64
tail -17 gpurun_out/stamps2.log
step bench_long 200 python -u bench.py
tail -1 gpurun_out/bench_long.log | cut -c1-200
step bench_driver 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_driver.log | cut -c1-200
step bench_driver2 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_driver2.log | cut -c1-200
