#!/bin/bash
# PMC passes over the direct 3x3 wgrad kernel (scripts/bench_wgrad3.py, one variant)
set -u
export TMPDIR=/tmp
D=gpurun_out/pmc_w3
mkdir -p $D
P1="SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  BENCH_W3_ONLY=${W3V:-s2w256} timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $D -o p$i -- python scripts/bench_wgrad3.py > $D/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo pmc-done
