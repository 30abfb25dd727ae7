#!/bin/bash
# Whisper bench with fp8 GEMM candidates left out (AIKO_FP8_SKIP), interleaved
set -o pipefail
export PYTHONPATH=.
for sk in none 256x256x4 128x256x5 256x256x3 none 256x256x4 128x256x5 256x256x3; do
  if [ "$sk" = none ]; then unset AIKO_FP8_SKIP; else export AIKO_FP8_SKIP=$sk; fi
  timeout -k 10 300 python -u bench.py --model whisper-small --steps 20 --warmup 5 > gpurun_out/skf_$sk.log 2>&1 || { tail -5 gpurun_out/skf_$sk.log; exit 1; }
  echo "whisper fp8 skip $sk: $(grep -o '"value": [0-9.]*' gpurun_out/skf_$sk.log)"
done
