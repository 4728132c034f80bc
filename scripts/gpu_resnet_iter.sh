#!/bin/bash
# ResNet-path iteration: native-graph / layer / op GPU tests, then the ResNet-18 bench x2
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_graph_gpu.py tests/test_native_layers_gpu.py tests/test_hip_ops_gpu.py tests/test_native_infer_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_rn.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_rn.log)"; [ $rc -le 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/rn_$i.log 2>&1 || exit $?
  echo "resnet: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn_$i.log)"
done
