#!/bin/bash
cd $GRAFT_REPO_ROOT
for m in 0 7 128 4 32; do for v in 0 1; do
  echo -n "rreg $v mode $m: "; AIKO_BN_RREG=$v AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 2>&1 | grep us/launch || exit 1
done; done
