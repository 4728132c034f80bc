#!/bin/bash
# A/B of the ResNet-18 step: BatchNorm statistics via fp64 accumulators finalized in the
# consumer kernels (DAMD_BN_FIN=1) vs per-block partials + finalize kernels (0).
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for f in 0 1; do
    DAMD_BN_FIN=$f timeout -k 10 200 python -u bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/ab_bnfin_$f.log 2>&1 || exit $?
    echo "BN_FIN=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bnfin_$f.log)"
  done
done
