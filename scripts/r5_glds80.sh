#!/bin/bash
# exact-N (BN = 80) LDS-DMA tiles: numerics, YOLO layer table and bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "test_conv" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python3 -u scripts/model_layers.py --model yolov8n --batch 64 > gpurun_out/layers_yolo_g80.txt 2>&1 || { tail -5 gpurun_out/layers_yolo_g80.txt; exit 1; }
grep -E "^ (46|48|51|53|56|58) " gpurun_out/layers_yolo_g80.txt; tail -1 gpurun_out/layers_yolo_g80.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
