#!/bin/bash
# A/B HIP runtime environment settings on both benches (driver flags); args = env settings
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for e in "$@"; do
  timeout -k 10 200 env $e python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/ab_rn.log 2>&1 || { tail -5 gpurun_out/ab_rn.log; exit 1; }
  timeout -k 10 200 env $e python -u bench.py --steps 20 --warmup 5 > gpurun_out/ab_mn.log 2>&1 || { tail -5 gpurun_out/ab_mn.log; exit 1; }
  echo "$e: rn $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_rn.log) mnist $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_mn.log)"
done
