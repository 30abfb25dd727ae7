#!/bin/bash
# Latency operating points: p50 / p99 per batch for ResNet-50 and YOLOv8-n
# at B = 1, 8, 32 (and the throughput batch), one frame in flight (--depth 0, --lanes 1: each
# batch's result is waited for before the next is submitted), hipGraph replay.
#   bash scripts/latency_table.sh > gpurun_out/latency.jsonl
set -o pipefail
for model in resnet50 yolov8n; do
  for b in 1 8 32; do
    timeout -k 10 120 python3 bench.py --model $model --batch $b --steps 200 --warmup 20 --depth 0 --lanes 1 \
      2>/dev/null | grep '^{' || exit 1
  done
done
