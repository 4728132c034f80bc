#!/bin/bash
# conv kernel iteration: conv GEMM / direct conv tests, direct-conv phase stamps on the
# ResNet-18 shapes, ResNet-18 bench
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gemm_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/t_conv.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/t_conv.log)"; [ $rc -le 1 ] || exit $rc
for a in "56 64 64" "56 64 64 dgrad" "28 128 128" "14 256 256" "14 256 256 dgrad"; do
  timeout -k 10 120 python -u scripts/stamps_conv3.py $a 2>&1 | grep -E "blocks|taps|block total" || exit 1
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model resnet18 --steps 30 --warmup 5 > gpurun_out/rn_$i.log 2>&1 || exit $?
  echo "resnet: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rn_$i.log)"
done
