#!/bin/bash
# Whisper-small bench: frame lanes
cd $GRAFT_REPO_ROOT
for i in 1 2; do for a in "--lanes 2" "--lanes 3" "--lanes 1"; do
  echo -n "[$a] "; timeout -k 10 400 python bench.py --model whisper-small --steps 20 --warmup 5 $a 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' '; echo
  [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
done; done
