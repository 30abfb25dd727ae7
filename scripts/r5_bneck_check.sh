#!/bin/bash
# bneck_fused: numerics (GPU tests), isolated timings old (AIKO_BN_RREG=0) vs new, bench A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for i in 1 2; do
for v in 0 1; do
  echo -n "rreg $v: "; AIKO_BN_RREG=$v timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 || exit 1
done; done
AIKO_BN_RREG=1 timeout -k 10 60 python scripts/bneck_run.py --grid 256 --stamps || exit 1
bash scripts/ab_multi.sh 3 AIKO_BN_RREG=0 AIKO_BN_RREG=1
