#!/bin/bash
# MNIST 1-GPU iteration: fused-engine GPU tests, phase stamps, benches (driver flags x2, long).
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fused_convnet_gpu.py -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fused.log 2>&1
rc=$?; echo "fused rc=$rc"; tail -2 gpurun_out/fused.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/fused.log | head -20; exit $rc; }
timeout -k 10 120 python -u scripts/stamps.py 64 > gpurun_out/stamps.log 2>&1; echo "stamps rc=$?"; cat gpurun_out/stamps.log | grep -v amdgpu
for r in 1 2; do timeout -k 10 100 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bq.log 2>&1 || exit 1; echo "drv $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bq.log)"; done
timeout -k 10 100 python -u bench.py --gpus 1 > gpurun_out/bql.log 2>&1 || exit 1; echo "long $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bql.log)"
