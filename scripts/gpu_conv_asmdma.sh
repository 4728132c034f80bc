#!/bin/bash
# LDS-DMA from inline asm: all conv-kernel numerics, then per-layer + wgrad3 sweeps, ResNet bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # run <name> <limit_s> <cmd...>
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -n 6
  [ $rc -eq 0 ] || exit $rc
}
run t_conv 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_native_graph_gpu.py
run t_w3_s4 200 env DAMD_WGRAD3_STAGES=4 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gemm_gpu.py -k direct_wgrad3
run bench_w3 300 python -u scripts/bench_wgrad3.py
run bench_gemm 300 env BENCH_CFG=0:2 python -u scripts/bench_gemm.py
run bench_resnet 300 python -u bench.py --model resnet18 --steps 20 --warmup 5
echo asmdma-done
