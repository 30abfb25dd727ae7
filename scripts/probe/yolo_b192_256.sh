#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for b in 192 256; do
    echo -n "yolo B=$b: "; timeout -k 10 240 python bench.py --model yolov8n --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
