#!/bin/bash
# packed-tap stem: conv kernel tests, then the native-graph suite + ResNet-18 bench A/B
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py -k "stem or subpixel" > gpurun_out/t_stem.log 2>&1 || { grep -v amdgpu gpurun_out/t_stem.log | tail -40; exit 1; }
tail -1 gpurun_out/t_stem.log
bash scripts/gpu_resnet_quick.sh DAMD_STEM4=0
