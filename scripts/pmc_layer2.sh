#!/bin/bash
# FETCH / WRITE sizes and wait cycles of one layer_bench layer for a few tiles:
#   scripts/pmc_layer2.sh <layer> <tile> [<tile> ...]
layer=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for tile in "$@"; do
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set -d $R/gpurun_out/pmcl2_${layer}_${tile//,/_}_$i -o run --output-format csv -- \
      python3 $R/scripts/layer_bench.py --layers $layer --iters 3 --tile $tile > /dev/null 2>&1 || exit 1
  done
  python3 $R/scripts/pmc_table.py $R/gpurun_out/pmcl2_${layer}_${tile//,/_}_* --top 1 | tail -1 | sed "s/^/$layer $tile /"
done
