#!/bin/bash
# ResNet bench: model switches A/B (chain kernels, stage-2 chain, MALL sub-batch chunking), interleaved
set -o pipefail
export PYTHONPATH=.
run() { env $1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/env_ab.log 2>&1 || { tail -5 gpurun_out/env_ab.log; exit 1; }
        echo "$1: $(grep -o '"value": [0-9.]*' gpurun_out/env_ab.log)"; }
for i in 1 2 3; do
  run "AIKO_NONE=1"
  run "AIKO_CHAIN2=0"
  run "AIKO_RESNET_CHAIN=0"
  run "AIKO_RESNET_MALL_CHUNK=80"
done
