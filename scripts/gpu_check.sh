#!/bin/bash
# One gpurun session: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
STAGE=${1:-all}
step() {  # step <name> <limit_s> <cmd...>   (stdout/err -> gpurun_out/<name>.log)
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s): $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
python -c "import torch;print(torch.cuda.get_device_name(0))"
if [ "$STAGE" = all ] || [ "$STAGE" = test ]; then
  step pytest_gpu 900 python -m pytest tests -q -m gpu -p no:cacheprovider
  step smoke 300 python __graft_entry__.py smoke
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  step stamps 300 python scripts/stamps.py 64
  step bench_n1 300 python bench.py --gpus 1 --steps 3000 --warmup 300
  step bench_n1_generic 300 python bench.py --gpus 1 --steps 200 --warmup 20 --engine generic
fi
if [ "$STAGE" = all ] || [ "$STAGE" = resnet ]; then
  step bench_gemm 300 python scripts/bench_gemm.py 64
  step bench_resnet 400 python bench.py --model resnet18 --steps 30 --warmup 5
  step rocprof_resnet 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o resnet -- python bench.py --model resnet18 --steps 10 --warmup 3
fi
if [ "$STAGE" = all ] || [ "$STAGE" = prof ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python bench.py --gpus 1 --steps 500 --warmup 50
fi
