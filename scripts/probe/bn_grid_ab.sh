#!/bin/bash
# stage-1 workgroup count (resnet50._BN_GRID) after the counted-wait fix, interleaved bench A/B
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for g in 0 224 192 160; do
    echo -n "grid $g: "
    timeout -k 10 300 python -c "
import sys
import aiko_services_amd.models.resnet50 as r
r._BN_GRID = $g
import bench
bench.main(['--steps', '20', '--warmup', '5'])" 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
