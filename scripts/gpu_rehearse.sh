#!/bin/bash
# Rehearse the driver's multi-GPU bench launch on ONE GPU: N ranks share cuda:0
# (control plane over gloo, per-step gradient all-reduce over the native peer kernel),
# plus the driver's short 1-GPU bench. Every GPU step has its own limit; a fault,
# abort or timeout stops the script.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <limit_s> <cmd...>   (stdout/err -> gpurun_out/<name>.log)
  local name=$1 lim=$2; shift 2
  echo "=== $name (limit ${lim}s): $*"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
step drv_n1 200 python bench.py --gpus 1 --steps 20 --warmup 5
step drv_n1_w40 200 python bench.py --gpus 1 --steps 20 --warmup 40
for N in ${RANKS:-2 4}; do
  DAMD_COMM=gloo step share_n$N 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 200 --warmup 20
done
echo rehearse-done
