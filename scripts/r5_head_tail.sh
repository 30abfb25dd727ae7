#!/bin/bash
# Detect-head class branch with the 1x1 fused into the 3x3's epilogue (conv_glds TAIL):
# numerics (all detect tests) and the YOLO bench with / without the box-branch tail (class tail on), interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_detect.py > gpurun_out/tail_test.log 2>&1 || { tail -30 gpurun_out/tail_test.log; exit 1; }
tail -2 gpurun_out/tail_test.log
for t in 1 0 1 0; do export AIKO_HEAD_TAIL_BOX=$t
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/tail_b$t.log 2>&1 || { tail -5 gpurun_out/tail_b$t.log; exit 1; }
  echo "HEAD_TAIL_BOX=$t $(grep -o '"value": [0-9.]*' gpurun_out/tail_b$t.log)"
done
