#!/bin/bash
# ResNet-50 bench sweep over per-step batch and lane count (frames/s, p50 latency)
cd $GRAFT_REPO_ROOT
for cfg in "256 2" "256 3" "256 4" "512 2" "512 4" "384 3"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --steps 30 --warmup 6 --batch $1 --lanes $2 > gpurun_out/bl_$1_$2.log 2>&1 || exit 1
  echo "batch $1 lanes $2: $(grep -o '"value": [0-9.]*' gpurun_out/bl_$1_$2.log) $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/bl_$1_$2.log)"
done
