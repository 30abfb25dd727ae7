#!/bin/bash
# 3x3 conv + following 1x1 in one conv_glds launch (TAIL: detect-head branches, l3 -> l4.cv1, l5 -> l6.cv1):
# numerics (all detect tests) and the YOLO bench with / without every tail fusion (AIKO_HEAD_TAIL), interleaved.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_detect.py > gpurun_out/tail_test.log 2>&1 || { tail -30 gpurun_out/tail_test.log; exit 1; }
tail -2 gpurun_out/tail_test.log
for t in 1 0 1 0; do export AIKO_HEAD_TAIL=$t
  timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/tail_b$t.log 2>&1 || { tail -5 gpurun_out/tail_b$t.log; exit 1; }
  echo "HEAD_TAIL=$t $(grep -o '"value": [0-9.]*' gpurun_out/tail_b$t.log)"
done
