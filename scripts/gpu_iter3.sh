#!/bin/bash
# iteration check: MNIST bench at the driver's flags (x3) and defaults, fused / peer tests
set -u
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_drv_$i.log 2>&1 || exit $?
  echo "driver flags run $i: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_drv_$i.log)"
done
timeout -k 10 200 python -u bench.py > gpurun_out/bench_def.log 2>&1 || exit $?
echo "defaults: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_def.log)"
timeout -k 10 600 python -u -m pytest tests/test_fused_convnet_gpu.py tests/test_peer_allreduce_gpu.py tests/test_dp_gpu.py -v -x --timeout 300 --timeout-method thread > gpurun_out/pytest_fused.log 2>&1; rc=$?; echo "fused/peer tests rc=$rc $(tail -1 gpurun_out/pytest_fused.log)"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
DAMD_COMM=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 400 --warmup 40 > gpurun_out/share_n2.log 2>&1; echo "shared N=2: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/share_n2.log) $(grep -o '"allreduce": "[a-z-]*"' gpurun_out/share_n2.log)"
DAMD_PEER_FOLD=0 DAMD_COMM=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 400 --warmup 40 > gpurun_out/share_n2_nofold.log 2>&1; echo "shared N=2 unfolded: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/share_n2_nofold.log)"
