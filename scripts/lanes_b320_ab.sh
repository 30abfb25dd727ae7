#!/bin/bash
# frame lanes at the B=320 default: interleaved ResNet-50 bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for l in 2 3 4; do
    echo -n "lanes=$l: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 --lanes $l 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
