#!/bin/bash
# per-kernel times of the Whisper bench, LN folded vs row-norm passes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 0; do
  AIKO_WHISPER_LN_FOLD=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lnprof$v -o run -- python3 bench.py --model whisper-small --steps 10 --warmup 3 > gpurun_out/lnprof$v.log 2>&1 || exit 1
  f=$(find gpurun_out/lnprof$v -name "*kernel_stats.csv" | head -1)
  echo "== ln_fold=$v"; head -14 "$f" | cut -d, -f1-4
done
