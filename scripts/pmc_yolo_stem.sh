#!/bin/bash
# PMC counter passes over the fused YOLO stem (scripts/yolo_stem_bench.py), one group per run
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 60 rocprofv3 --pmc $set -d $R/gpurun_out/pmc_ystem_${i} -o run --output-format csv -- \
    python3 $R/scripts/yolo_stem_bench.py 64 5 > /dev/null 2>&1 || exit $?
done
