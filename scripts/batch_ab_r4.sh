#!/bin/bash
# Round-4 kernel mix: headline bench at batch sizes around the B=320 default, interleaved (driver shape).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for b in ${BATCHES:-320 384 448 512}; do
    echo -n "B=$b: "; timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch $b 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
