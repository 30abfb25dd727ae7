#!/bin/bash
# PMC counter passes over one layer_bench layer/tile: scripts/pmc_layer.sh <layer> <tile> <tag>
layer=$1; tile=$2; tag=$3
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set -d $R/gpurun_out/pmcl_${tag}_${i} -o run --output-format csv -- \
    python3 $R/scripts/layer_bench.py --layers $layer --iters 3 --tile $tile || exit $?
done
