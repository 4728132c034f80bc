#!/bin/bash
# native-graph engine tests + ResNet-18 bench (+ A/B env given as arguments)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_native_graph_gpu.py tests/test_dp_gpu.py > gpurun_out/t_ng.log 2>&1 || { tail -30 gpurun_out/t_ng.log; exit 1; }
tail -1 gpurun_out/t_ng.log
timeout -k 10 200 python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/b_rn.log 2>&1 || { tail -20 gpurun_out/b_rn.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_rn.log
for e in "$@"; do
  timeout -k 10 200 env $e python -u bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/b_rn_ab.log 2>&1 || { tail -20 gpurun_out/b_rn_ab.log; exit 1; }
  echo "$e: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/b_rn_ab.log)"
done
