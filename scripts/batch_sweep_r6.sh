#!/bin/bash
# round 6: larger batches for configs 4 / 5 (interleaved, two rounds, driver-shaped runs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for b in 64 128 192; do
    echo -n "yolo B=$b: "; timeout -k 10 240 python bench.py --model yolov8n --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
  for b in 14 28 42; do
    echo -n "whisper streams=$b: "; timeout -k 10 300 python bench.py --model whisper-small --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
