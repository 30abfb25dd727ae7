#!/bin/bash
# Persistent fp8 GEMM (tuner variant 4) at the Whisper qkv / fc1 shapes: numerics tests, then
# timings under AIKO_FP8_DIAG switches (1: no K-block DMAs after the first two, 2: no epilogue
# stores, 4: no per-block barrier).  Timing diagnostics only: non-zero bits give wrong results.
set -o pipefail
for a in ${OVS:-1}; do
  AIKO_FP8_OVERLAP=$a timeout -k 10 120 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_transformer.py -k "persistent" || exit 1
done
for op in gemm_qkv gemm_fc1; do
  for a in ${OVS:-1}; do
    for d in ${DIAGS:-0 3 7}; do
      echo -n "$op overlap=$a diag=$d: "
      AIKO_FP8_OVERLAP=$a AIKO_FP8_DIAG=$d timeout -k 10 90 python scripts/op_bench.py $op --batch 14 --tile 256,256,4 --iters 50 --reps 5 2>&1 | grep "TFLOP" || exit 1
    done
  done
done
# Whisper-small encoder bench (14 streams) A/B over the overlap switch, interleaved
for i in $(seq ${WHISPER_AB:-0}); do
  for a in 0 1; do
    echo -n "whisper overlap=$a: "
    AIKO_FP8_OVERLAP=$a timeout -k 10 300 python bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
