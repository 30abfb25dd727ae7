#!/bin/bash
# bneck_fused ablation timings (AIKO_BN_MODE bits, see bneck_fused.hip) + per-phase stamps
cd $GRAFT_REPO_ROOT
for m in 0 128 32 7 135 1 2 4 16; do
  echo -n "mode $m: "; AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 || exit 1
done
echo -n "dual mode 0: "; timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --dual || exit 1
timeout -k 10 60 python scripts/bneck_run.py --grid 256 --stamps || exit 1
