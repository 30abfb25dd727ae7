#!/bin/bash
# variant 20 (persistent conv_wide) in / out of tuning: YOLO and Whisper benches, interleaved
set -o pipefail
export PYTHONPATH=.
for sk in none 20 none 20; do
  if [ "$sk" = none ]; then unset AIKO_CONV_SKIP; else export AIKO_CONV_SKIP=$sk; fi
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/s20y_$sk.log 2>&1 || { tail -5 gpurun_out/s20y_$sk.log; exit 1; }
  echo "yolo skip $sk: $(grep -o '"value": [0-9.]*' gpurun_out/s20y_$sk.log)"
done
for sk in none 20; do
  if [ "$sk" = none ]; then unset AIKO_CONV_SKIP; else export AIKO_CONV_SKIP=$sk; fi
  timeout -k 10 300 python -u bench.py --model whisper-small --steps 20 --warmup 5 > gpurun_out/s20w_$sk.log 2>&1 || { tail -5 gpurun_out/s20w_$sk.log; exit 1; }
  echo "whisper skip $sk: $(grep -o '"value": [0-9.]*' gpurun_out/s20w_$sk.log)"
done
