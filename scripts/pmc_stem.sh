#!/bin/bash
# PMC counter passes over the fused stem+pool kernel: scripts/pmc_stem.sh [batch]
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B=${1:-64}
i=0
for set in "SQ_WAVES SQ_LEVEL_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d $R/gpurun_out/pmcs2_${i} -o run --output-format csv -- \
    python3 $R/scripts/stem_pool_bench.py $B || exit $?
done
