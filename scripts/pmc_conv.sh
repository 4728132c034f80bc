#!/bin/bash
# PMC passes over one direct-conv launch mode on one ResNet-18 shape:
#   CONV="56 64 64 fwd" bash scripts/pmc_conv.sh   -> gpurun_out/pmc_conv_<tag>/
set -u
export TMPDIR=/tmp
TAG=${TAG:-c}
D=gpurun_out/pmc_conv_$TAG
mkdir -p $D
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D/p$i -o p$i -- python3 scripts/conv3_run.py ${CONV:-56 64 64 fwd} > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
python3 scripts/pmc_csv.py $D conv wgrad > $D/summary.txt
echo pmc-done $TAG
