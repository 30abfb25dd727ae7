#!/bin/bash
# YOLOv8-n bench: frame lanes / batches in flight
cd $GRAFT_REPO_ROOT
for i in 1 2; do for a in "--lanes 2" "--lanes 3" "--lanes 2 --depth 3"; do
  echo -n "[$a] "; timeout -k 10 300 python bench.py --model yolov8n --steps 30 --warmup 6 $a 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' '; echo
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done; done
