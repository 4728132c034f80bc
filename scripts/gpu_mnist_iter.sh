#!/bin/bash
# MNIST step iteration: fused-engine GPU tests, phase stamps, bench at the driver's flags
# (x2) and defaults
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_convnet_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_mnist.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_mnist.log)"; [ $rc -le 1 ] || exit $rc
if [ "${STAMPS:-1}" = 1 ]; then
  timeout -k 10 120 python -u scripts/stamps.py 64 > gpurun_out/stamps.log 2>&1 || exit $?
  grep -E "^fwd|^bwd|^ +[0-9] " gpurun_out/stamps.log
fi
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$i.log 2>&1 || exit $?
  echo "driver flags: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_drv_$i.log)"
done
DAMD_BENCH_FINAL_GRAPH=0 timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_nofinal.log 2>&1 || exit $?
echo "driver flags, no final graph: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_drv_nofinal.log)"
timeout -k 10 200 python -u bench.py > gpurun_out/bench_def.log 2>&1 || exit $?
echo "defaults: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_def.log)"
