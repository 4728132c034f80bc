#!/bin/bash
# iteration check after a change to both steps: native / conv GPU tests, fused tests,
# MNIST stamps + benches, ResNet bench, conv3 stamps
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_native_graph_gpu.py tests/test_native_layers_gpu.py tests/test_native_infer_gpu.py tests/test_hip_ops_gpu.py tests/test_conv_gemm_gpu.py tests/test_fused_convnet_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_iter4.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_iter4.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u scripts/stamps.py 64 > gpurun_out/stamps.log 2>&1 || exit $?
grep -E "fwd|bwd|loads|staged|conv done|atomics|head|end" gpurun_out/stamps.log | head -14
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$i.log 2>&1 || exit $?
  echo "driver flags: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_drv_$i.log)"
done
timeout -k 10 200 python -u bench.py > gpurun_out/bench_def.log 2>&1 || exit $?
echo "defaults: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_def.log)"
timeout -k 10 200 python -u bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/rn.log 2>&1 || exit $?
echo "resnet: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn.log)"
for a in "56 64 64" "56 64 64 dgrad" "28 128 128" "14 256 256"; do timeout -k 10 120 python -u scripts/stamps_conv3.py $a 2>&1 | grep -v amdgpu.ids || exit 1; done
