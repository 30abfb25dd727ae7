#!/bin/bash
# Timing ablation of the fused bottleneck: AIKO_BN_MODE bits drop parts of the loop
# (1 conv2, 2 conv1, 4 conv3, 8 DMA waits, 16 barriers, 32 DMAs, 64 L2 touches).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for m in 0 128 4 40 168 132 ${MODES:-}; do
  echo "mode $m: $(AIKO_BN_MODE=$m timeout -k 5 60 python3 $R/scripts/bneck_run.py --time "$@" 2>&1 | tail -1)"
done
