#!/bin/bash
# Iteration check: selected GPU test files (args, default: conv/ops/native-graph/fused),
# then the MNIST bench with the driver's flags and the ResNet-18 bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TESTS:-tests/test_conv_gemm_gpu.py tests/test_hip_ops_gpu.py tests/test_native_graph_gpu.py tests/test_fused_convnet_gpu.py}
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread $T > gpurun_out/it_tests.log 2>&1
rc=$?; tail -3 gpurun_out/it_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/it_tests.log | head -20; exit $rc; }
timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/it_mnist.log 2>&1 || { tail -20 gpurun_out/it_mnist.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/it_mnist.log
timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/it_rn.log 2>&1 || { tail -20 gpurun_out/it_rn.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/it_rn.log
if [ -n "${PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_it -o resnet -- python3 bench.py --model resnet18 --steps 10 --warmup 3 > gpurun_out/prof_it.log 2>&1 || exit 1
fi
