#!/bin/bash
# config 3 (pp, world 1): batch 320 vs 640, interleaved
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for b in 320 640; do
    echo -n "pp B=$b: "; timeout -k 10 300 python bench.py --parallel pp --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
