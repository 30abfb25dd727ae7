#!/bin/bash
# fp8 GEMM tile/variant sweep at Whisper-small shapes (B=16 clips of 30 s)
for op in gemm_qkv gemm_out gemm_fc1 gemm_fc2; do
  for t in 128,128,0 128,128,1 128,64,0 128,64,1 64,128,0 64,128,1 64,64,0 64,64,1; do
    python scripts/op_bench.py $op --tile $t || exit $?
  done
done
