#!/bin/bash
cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 60 python scripts/yolo_stem_bench.py 64 200 2>&1 | grep -v amdgpu || exit 1
  AIKO_STEM_FAST_WIDE=0 timeout -k 10 60 python scripts/yolo_stem_bench.py 64 200 2>&1 | grep -v amdgpu || exit 1
done
bash scripts/r3_benches.sh || exit 1
for w in none fc stem gap; do
  echo -n "sensitivity $w: "
  timeout -k 10 200 python scripts/sensitivity.py $w --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
