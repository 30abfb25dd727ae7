#!/bin/bash
# interleaved A/B of the default ResNet bench against several env settings:
#   scripts/probe/ab_multi_env.sh rounds "ENV=VAL" "ENV=VAL ENV2=VAL" ...
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
N=$1; shift
for i in $(seq $N); do
  echo -n "default: "; timeout -k 10 240 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  for e in "$@"; do
    echo -n "$e: "; env $e timeout -k 10 240 python bench.py --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
