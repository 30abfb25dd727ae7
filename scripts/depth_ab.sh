#!/bin/bash
# batches in flight x frame lanes at B=320: interleaved ResNet-50 bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for cfg in "--lanes 2 --depth 2" "--lanes 2 --depth 3" "--lanes 3 --depth 3" "--lanes 4 --depth 4"; do
    echo -n "$cfg: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 $cfg 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
