#!/bin/bash
# PMC passes over the conv GEMMs of one layer (each pass its own rocprofv3 run).
set -u
export TMPDIR=/tmp
L="$*"
D=gpurun_out/pmc
mkdir -p $D
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D -o p$i -- python scripts/gemm_one.py $L 5 > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc-done
