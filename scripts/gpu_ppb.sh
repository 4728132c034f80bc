#!/bin/bash
# A/B of the backward kernel's slicing (DAMD_PP_BWD): kernel durations under rocprofv3
# (stable) and interleaved short benches.
export TMPDIR=/tmp; mkdir -p gpurun_out
for ppb in 1 2 3; do
  DAMD_PP_BWD=$ppb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ppb$ppb -o p -- python3 bench.py --gpus 1 --steps 500 --warmup 50 > gpurun_out/ppb_prof$ppb.log 2>&1
  echo "prof ppb=$ppb rc=$?"
  f=$(find gpurun_out/ppb$ppb -name "*kernel_stats.csv" | head -1); grep -E "convnet2" $f | cut -d, -f1-8 | head -4
done
for rep in 1 2; do for ppb in 1 2 3; do
  DAMD_PP_BWD=$ppb timeout -k 10 100 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ppbb.log 2>&1 || exit 1
  echo "ppb=$ppb rep=$rep $(tail -1 gpurun_out/ppbb.log | grep -o '"ms_per_step": [0-9.]*')"
done; done
