#!/bin/bash
# rocprofv3 kernel traces of both benchmark steps (headline MNIST CNN, ResNet-18) at HEAD.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mnist -o bench -- python3 bench.py --gpus 1 --steps 500 --warmup 50 > gpurun_out/prof_mnist.log 2>&1 || { tail -5 gpurun_out/prof_mnist.log; exit 1; }
tail -1 gpurun_out/prof_mnist.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet_r2 -o resnet -- python3 bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/prof_resnet_r2.log 2>&1 || { tail -5 gpurun_out/prof_resnet_r2.log; exit 1; }
tail -1 gpurun_out/prof_resnet_r2.log
