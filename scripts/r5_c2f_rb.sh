#!/bin/bash
# fused C2f band height sweep (YOLOv8-n bench)
cd $GRAFT_REPO_ROOT
for i in 1 2; do for rb in 32 40 80 160; do
  echo -n "rb $rb: "; AIKO_C2F_RB=$rb timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done; done
