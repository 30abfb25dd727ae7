#!/bin/bash
# exact-N 144 LDS-DMA tiles for YOLO's first head conv: numerics, layer table, bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "igemm or glds or exact" > gpurun_out/g144_test.log 2>&1 || { tail -30 gpurun_out/g144_test.log; exit 1; }
tail -1 gpurun_out/g144_test.log
timeout -k 10 300 python3 -u scripts/model_layers.py --model yolov8n --batch 64 > gpurun_out/g144_layers.txt 2>&1 || { tail -5 gpurun_out/g144_layers.txt; exit 1; }
grep -E " (28|29|30) M=|whole" gpurun_out/g144_layers.txt
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/g144_b.log 2>&1 || { tail -5 gpurun_out/g144_b.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/g144_b.log
done
