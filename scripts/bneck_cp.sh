#!/bin/bash
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for i in 1 2; do for v in 0 1 2 3; do
  echo -n "cp $v: "; AIKO_BN_CP=$v timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 2>&1 | grep us/ || exit 1
  echo -n "cp $v dual: "; AIKO_BN_CP=$v timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --dual 2>&1 | grep us/ || exit 1
done; done
bash scripts/ab_multi.sh 2 AIKO_BN_CP=0 AIKO_BN_CP=1 AIKO_BN_CP=2 AIKO_BN_CP=3
