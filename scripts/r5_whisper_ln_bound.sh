#!/bin/bash
# upper bound of removing the LayerNorm passes: Whisper-small bench with / without them (timing only)
cd $GRAFT_REPO_ROOT
for i in 1 2; do for v in 0 1; do
  echo -n "skip_ln=$v: "; AIKO_WHISPER_DIAG_SKIP_LN=$v timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done; done
