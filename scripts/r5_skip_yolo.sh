#!/bin/bash
# YOLO bench with tuner variants left out (AIKO_CONV_SKIP), interleaved
set -o pipefail
export PYTHONPATH=.
for sk in none 9 2 12 3 8 none 9 2 12 3 8; do
  if [ "$sk" = none ]; then unset AIKO_CONV_SKIP; else export AIKO_CONV_SKIP=$sk; fi
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/sky_$sk.log 2>&1 || { tail -5 gpurun_out/sky_$sk.log; exit 1; }
  echo "yolo skip $sk: $(grep -o '"value": [0-9.]*' gpurun_out/sky_$sk.log)"
done
