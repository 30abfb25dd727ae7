#!/bin/bash
# Persistent fp8 GEMM variants 4 / 5: numerics, then isolated timings at the Whisper-small
# 14-stream shapes and the bench with the tuner's picks printed.
set -o pipefail
export AIKO_FP8_V4MX=${AIKO_FP8_V4MX:-1}
timeout -k 10 180 python -u -m pytest -x -q --timeout 90 --timeout-method thread tests/test_gpu_transformer.py -k "persistent or mx_in" || exit 1
run() { echo -n "$1 $2: "; timeout -k 10 90 python scripts/op_bench.py $1 --batch 14 --tile $2 --iters 50 --reps 5 2>&1 | grep "TFLOP" || echo "(n/a)"; }
run out_mxr 256,256,3; run out_mxr 128,256,5; run out_mxr 256,256,4
run fc2_mxr 256,256,3; run fc2_mxr 128,256,5; run fc2_mxr 256,256,4
for i in 1 2; do
  echo -n "whisper default: "
  timeout -k 10 300 python bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
AIKO_TUNE_VERBOSE=1 timeout -k 10 300 python bench.py --model whisper-small --steps 2 --warmup 1 2>&1 | grep "tune fp8" | sort | uniq | head -20
