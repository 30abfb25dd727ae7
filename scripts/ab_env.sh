#!/bin/bash
# interleaved A/B of the ResNet bench: scripts/ab_env.sh "<ENV=VAL ...>" [rounds]
cd $GRAFT_REPO_ROOT
B="$1"; N=${2:-3}
for i in $(seq $N); do
  echo -n "A default: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  echo -n "B $B: "; env $B timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
