#!/bin/bash
# letterbox + stem + l1 in one launch: numerics (all detect tests) and the YOLO bench A/B
set -o pipefail
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_detect.py > gpurun_out/sl_test.log 2>&1 || { tail -40 gpurun_out/sl_test.log; exit 1; }
tail -1 gpurun_out/sl_test.log
for t in 1 0 1 0 1 0; do
  AIKO_STEM_L1=$t timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/sl_b$t.log 2>&1 || { tail -5 gpurun_out/sl_b$t.log; exit 1; }
  echo "STEM_L1=$t $(grep -o '"value": [0-9.]*' gpurun_out/sl_b$t.log)"
done
