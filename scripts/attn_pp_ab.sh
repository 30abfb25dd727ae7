#!/bin/bash
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for v in 0 15; do echo -n "variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 60 python scripts/op_bench.py attn --iters 50 --reps 7 | grep attn: || exit 1; done
done
