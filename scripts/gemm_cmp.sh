#!/bin/bash
# fp8 GEMM variants at Whisper-small shapes: register-staged, 2-slot LDS-DMA, 8-wave LDS-DMA
for op in gemm_qkv gemm_out gemm_fc1 gemm_fc2; do
  for t in ${TILES:-128,128,0 128,128,1 256,128,2}; do
    echo -n "$t  "; python scripts/op_bench.py $op --tile $t 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
