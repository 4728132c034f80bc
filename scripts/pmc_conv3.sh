#!/bin/bash
# PMC passes over the direct 3x3 conv kernel on one ResNet-18 shape (scripts/stamps_conv3.py
# runs it 11 times); CONV3_SHAPE="h cin cout [dgrad]", default the layer-3 forward
set -u
export TMPDIR=/tmp
D=gpurun_out/pmc_c3
mkdir -p $D
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D -o p$i -- python scripts/stamps_conv3.py ${CONV3_SHAPE:-14 256 256} > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc-done
