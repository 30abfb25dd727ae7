#!/bin/bash
# PMC passes over the fused stage-1 bottleneck alone (scripts/bneck_run.py):
#   scripts/bneck_pmc.sh <tag> [bneck_run args] -> gpurun_out/pmcbn_<tag>_<pass>/ + table
tag=${1:-bn}
shift || true
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
i=0
dirs=""
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcbn_${tag}_${i} -o run --output-format csv -- \
    python3 $R/scripts/bneck_run.py "$@" > /dev/null 2>&1 || exit $?
  dirs="$dirs $R/gpurun_out/pmcbn_${tag}_${i}"
done
python3 $R/scripts/pmc_table.py $dirs --top 4 --lds | tee $R/gpurun_out/pmcbn_${tag}.md
