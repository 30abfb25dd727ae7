#!/bin/bash
# PMC counter passes over the headline bench (lanes=1 so dispatches do not overlap):
#   scripts/pmc_bench.sh <tag> [bench args]   -> gpurun_out/pmcb_<tag>_<pass>/
# One pass per counter group (rocprofv3 does not split counters over passes).
tag=${1:-r2}
shift || true
extra="$*"          # extra bench.py arguments, e.g. --model yolov8n
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $R/gpurun_out/pmcb_${tag}_${i} -o run --output-format csv -- \
    python3 $R/bench.py --steps 3 --warmup 2 --lanes 1 $extra > /dev/null 2>&1 || exit $?
done
