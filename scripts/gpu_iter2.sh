#!/bin/bash
# iteration check: MNIST bench at the driver's flags (x3) and defaults, fused-engine tests,
# ResNet BN_FIN A/B
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$i.log 2>&1 || exit $?
  echo "driver flags run $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_drv_$i.log)"
done
timeout -k 10 200 python -u bench.py > gpurun_out/bench_def.log 2>&1 || exit $?
echo "defaults: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_def.log)"
timeout -k 10 400 python -u -m pytest tests/test_fused_convnet_gpu.py tests/test_bench_cpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1; echo "fused tests rc=$? $(tail -1 gpurun_out/pytest_fused.log)"
bash scripts/ab_bnfin.sh
