#!/bin/bash
# 2-launch MNIST step: GPU tests of the fused engine + peer all-reduce, phase stamps,
# driver-flag and long benches, and a rocprofv3 kernel-stats pass.  Stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -60 "gpurun_out/$name.log"; exit $rc; fi
}
step t_fused 400 python -u -m pytest tests/test_fused_convnet_gpu.py -x -v -s -p no:cacheprovider --timeout 120 --timeout-method thread
grep -E "passed|failed|rel err|reference:" gpurun_out/t_fused.log | tail -20
step stamps2 120 python -u scripts/stamps.py 64
tail -16 gpurun_out/stamps2.log
step bench_drv 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_drv.log
step bench_long 200 python -u bench.py
tail -1 gpurun_out/bench_long.log
step t_peer 400 python -u -m pytest tests/test_peer_allreduce_gpu.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread
grep -E "passed|failed|us per" gpurun_out/t_peer.log | tail -5
