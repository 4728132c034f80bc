#!/bin/bash
# Round-4 profile set at HEAD: rocprofv3 kernel traces of the 1-GPU MNIST bench, of the
# N=2 rehearsal (two ranks sharing the GPU, sharded exchange inside the step kernels), of
# the ResNet-18 bench; in-kernel phase stamps; the benches at the driver's flags.  Each
# GPU step has its own limit; the first failure stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi
}
step prof_mnist 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_mnist -o bench -- python3 bench.py --gpus 1 --steps 500 --warmup 50
step stamps 120 python -u scripts/stamps.py 64
DAMD_COMM=gloo step prof_mnist_dp 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_mnist_dp -o dp -- python3 bench.py --gpus 2 --steps 50 --warmup 10
step prof_resnet 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_resnet -o resnet -- python3 bench.py --model resnet18 --steps 10 --warmup 3
step bench_driver 200 python -u bench.py --gpus 1 --steps 20 --warmup 5
tail -1 gpurun_out/bench_driver.log | cut -c1-220
step bench_long 200 python -u bench.py --phases 50
tail -1 gpurun_out/bench_long.log | cut -c1-220
step bench_resnet 300 python -u bench.py --model resnet18 --steps 20 --warmup 5
tail -1 gpurun_out/bench_resnet.log | cut -c1-220
