#!/bin/bash
# YOLOv8-n / Whisper-small at their default batches: frame lanes x batches in flight, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for m in yolov8n whisper-small; do
    for a in "--lanes 2 --depth 2" "--lanes 3 --depth 2" "--lanes 2 --depth 3" "--lanes 3 --depth 3"; do
      echo -n "$m $a: "; timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 $a 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
      echo
    done
  done
done
