#!/bin/bash
# split-KV tail experiments: no split / mapping only (s=1) / s=2,3,4,8 (repeated, interleaved)
cd $GRAFT_REPO_ROOT
run() { echo -n "$* : "; env "$@" timeout -k 10 60 python scripts/op_bench.py attn --iters 50 --reps 7 | grep attn: || exit 1; }
for rep in 1 2; do
  run AIKO_ATTN_WS=0
  run AIKO_ATTN_SPLIT_S=1
  run AIKO_ATTN_SPLIT_S=2
  run AIKO_ATTN_SPLIT_S=3
  run AIKO_ATTN_SPLIT_S=4
  run AIKO_ATTN_SPLIT_S=8
done
