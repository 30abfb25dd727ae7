#!/bin/bash
# Infinity-Cache blocking of the stem + stage-1 bottlenecks (AIKO_RESNET_MALL_CHUNK) on the
# round-4 fused bottleneck kernel, interleaved with the default, driver-shaped bench.
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for c in 0 ${MALL_CHUNKS:-64 80 160}; do
    echo -n "chunk $c: "
    AIKO_RESNET_MALL_CHUNK=$c timeout -k 10 200 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
