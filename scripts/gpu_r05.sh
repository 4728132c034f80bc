#!/bin/bash
# Round-5 GPU checks, stage by stage (STAGES="tests rehearse bench ..." selects).  Every GPU
# step has its own time limit; a fault, abort or timeout stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <limit_s> <cmd...>   (stdout/err -> gpurun_out/<name>.log)
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s): $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STAGES:-xtests bench}; do
  case $s in
    xtests)  # the exchange: in-process sharded ranks, bitwise cross-transport, self-test fallback
      step xtests 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
        tests/test_sharded_inproc_gpu.py tests/test_peer_allreduce_gpu.py ;;
    bn)  # BatchNorm fixed-point statistics
      step bntests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
        tests/test_hip_ops_gpu.py tests/test_conv_gemm_gpu.py -k "bn or bnin" ;;
    tests)
      step gputests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    bench)
      step bench_n1 200 python bench.py --gpus 1 --steps 20 --warmup 5
      step bench_n1_long 200 python bench.py --gpus 1 --steps 2000 --warmup 200 ;;
    rehearse)  # the driver's multi-GPU launch, N ranks sharing cuda:0 (gloo control plane)
      for N in ${RANKS:-2}; do
        DAMD_COMM=gloo step share_n$N 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
          --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 200 --warmup 20
      done ;;
    resnet)
      step resnet 300 python bench.py --model resnet18 --steps 20 --warmup 5 ;;
  esac
done
echo stages-done
