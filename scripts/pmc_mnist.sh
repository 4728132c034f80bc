#!/bin/bash
# PMC passes over the fused MNIST step (one counter group per run, --kernel-trace only):
# issue mix and wait cycles of the fwd / bwd kernels.  GPU box:  bash scripts/pmc_mnist.sh
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
OUT=gpurun_out/pmc_mnist
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
run() {  # run <name> <counters...>
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $OUT/$name -o run -- \
    python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE &&
run p2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM &&
python3 scripts/pmc_summary.py $OUT > $OUT/summary.txt 2>&1
echo "pmc done rc=$?"
