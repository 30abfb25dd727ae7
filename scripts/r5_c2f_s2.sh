#!/bin/bash
# l1 + l2 fused: numerics, YOLO tests, bench A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for i in 1 2; do for v in 1 0; do
  echo -n "s2=$v: "; AIKO_C2F_S2=$v timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done; done
