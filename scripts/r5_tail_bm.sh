#!/bin/bash
# tail-fusion tiles: 64-row (AIKO_TAIL_BM=64) vs 128-row: numerics and YOLO bench, interleaved
set -o pipefail
export PYTHONPATH=.
AIKO_TAIL_BM=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_detect.py -k "tail" > gpurun_out/tbm_test.log 2>&1 || { tail -30 gpurun_out/tbm_test.log; exit 1; }
tail -1 gpurun_out/tbm_test.log
for b in 64 128 64 128; do
  AIKO_TAIL_BM=$b timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/tbm_$b.log 2>&1 || { tail -5 gpurun_out/tbm_$b.log; exit 1; }
  echo "TAIL_BM=$b $(grep -o '"value": [0-9.]*' gpurun_out/tbm_$b.log)"
done
