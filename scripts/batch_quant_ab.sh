#!/bin/bash
# Batch sizes whose stage-3/4 tile counts fill 256 CUs (B=320: stage-3 M = 62720 = 245 x 256)
# against the B=256 default (196 tiles): interleaved ResNet-50 bench A/B.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for b in 256 320 640; do
    echo -n "B=$b: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
