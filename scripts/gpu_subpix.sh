#!/bin/bash
set -u
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_native_graph_gpu.py > gpurun_out/t_sp.log 2>&1 || { grep -v amdgpu gpurun_out/t_sp.log | tail -30; exit 1; }
tail -1 gpurun_out/t_sp.log
timeout -k 10 300 env BENCH_CFG=0:2 python -u scripts/bench_gemm.py > gpurun_out/bench_sp.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/bench_sp.log
bash scripts/gpu_resnet_quick.sh DAMD_DGRAD_SUBPIX=0 2>&1 | tail -3
