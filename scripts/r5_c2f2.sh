#!/bin/bash
# fused C2f on l2 and l15: numerics, band sweep for the 80-row block, bench
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for rb in 10 20 40; do
  echo -n "rb80 $rb: "; AIKO_C2F_RB80=$rb timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
