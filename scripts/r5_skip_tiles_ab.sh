#!/bin/bash
# ResNet bench with single tiles left out of tuning (AIKO_CONV_SKIP_TILES), interleaved
set -o pipefail
export PYTHONPATH=.
for sk in none 256x256x8 256x128x8 none 256x256x8 256x128x8 none 256x256x8 256x128x8; do
  if [ "$sk" = none ]; then unset AIKO_CONV_SKIP_TILES; else export AIKO_CONV_SKIP_TILES=$sk; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/skt_$sk.log 2>&1 || { tail -5 gpurun_out/skt_$sk.log; exit 1; }
  echo "skip tiles $sk: $(grep -o '"value": [0-9.]*' gpurun_out/skt_$sk.log)"
done
