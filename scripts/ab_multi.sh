#!/bin/bash
# interleaved A/B/C... of the ResNet bench: scripts/ab_multi.sh ROUNDS "<ENV=VAL ...>" "<ENV=VAL ...>" ...
# ("-" = defaults).  Extra bench flags via BENCH_ARGS.
cd $GRAFT_REPO_ROOT
N=$1; shift
for i in $(seq $N); do
  for v in "$@"; do
    e="$v"; [ "$e" = "-" ] && e=""
    echo -n "[$v] "; env $e timeout -k 10 200 python bench.py --steps 30 --warmup 6 $BENCH_ARGS 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' ; echo
    [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
  done
done
