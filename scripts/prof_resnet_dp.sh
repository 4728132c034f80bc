#!/bin/bash
# rocprofv3 kernel trace of the ResNet-18 bench at N = 2 ranks SHARING one GPU (DAMD_COMM=gloo:
# the native graph engine's gradient buckets go through the xGMI peer kernel on the side
# stream), to check that bucket all-reduces overlap the rest of backward.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${PROF_OUT:-gpurun_out/prof_rn_dp}
DAMD_COMM=gloo timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT -o rn -- \
  python3 bench.py --model resnet18 --gpus 2 --steps 10 --warmup 3 > $OUT.log 2>&1
rc=$?; tail -2 $OUT.log; exit $rc
