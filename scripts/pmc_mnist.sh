#!/bin/bash
# PMC pass over the MNIST step kernels: busy GPU cycles (clock), wave cycles, MFMA/VALU/LDS
# activity.  One counter group per run (rocprofv3 does not split passes).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_mnist
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pmc_mnist -o p1 -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/pmc_mnist/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc_mnist -o p2 -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/pmc_mnist/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc_mnist -o kt -- python3 bench.py --steps 500 --warmup 50 > gpurun_out/pmc_mnist/kt.log 2>&1
