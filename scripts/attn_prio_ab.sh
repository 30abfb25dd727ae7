#!/bin/bash
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for pr in 0 1; do echo -n "prio=$pr: "; AIKO_ATTN_PRIO=$pr timeout -k 10 60 python scripts/op_bench.py attn --iters 50 --reps 7 | grep attn: || exit 1; done
done
