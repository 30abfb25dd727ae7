#!/bin/bash
# isolated kernel numbers (median of 7 x 50 launches) for attention and the Whisper fp8 GEMMs
cd $GRAFT_REPO_ROOT
for op in attn gemm_qkv gemm_fc1 fc1_gelu_mx gemm_fc2 gemm_out; do
  timeout -k 10 120 python scripts/op_bench.py $op --iters 50 --reps 7 | grep -v amdgpu || exit 1
done
