#!/bin/bash
# batch / stream-count sweep for configs 4 (YOLOv8-n) and 5 (Whisper-small encoder)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for b in 12 14 16 20 24; do
    echo -n "whisper streams=$b: "; timeout -k 10 200 python bench.py --model whisper-small --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
for i in 1 2; do
  for b in 48 64 80 96; do
    echo -n "yolo B=$b: "; timeout -k 10 200 python bench.py --model yolov8n --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
