#!/bin/bash
# rocprofv3 kernel stats of the ResNet-18 bench step (1 GPU)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
OUT=${PROF_OUT:-gpurun_out/prof_resnet5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o resnet -- python bench.py --model resnet18 --steps 10 --warmup 3 > $OUT.log 2>&1
rc=$?; tail -2 $OUT.log; exit $rc
