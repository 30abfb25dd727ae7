#!/bin/bash
# ResNet bench: batches in flight (--depth) A/B, interleaved
set -o pipefail
export PYTHONPATH=.
for d in 2 3 4 2 3 4; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --depth $d > gpurun_out/depth_$d.log 2>&1 || { tail -5 gpurun_out/depth_$d.log; exit 1; }
  echo "depth $d: $(grep -o '"value": [0-9.]*' gpurun_out/depth_$d.log) $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/depth_$d.log)"
done
