#!/bin/bash
# L2 hit rate of the conv GEMM kernels of one ResNet-18 layer (rocprofv3 --pmc, one pass):
# usage: pmc_l2.sh h cin cout k s [tag]
set -u
export TMPDIR=/tmp
D=gpurun_out/pmc_l2
mkdir -p $D
TAG=${6:-l}
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $D -o $TAG -- python scripts/gemm_one.py $1 $2 $3 $4 $5 5 > $D/$TAG.log 2>&1 || { echo "pmc pass failed rc=$?"; exit 1; }
echo pmc-done
