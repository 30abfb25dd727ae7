#!/bin/bash
# End-of-round-3 ResNet-50 profile at the B=320 default: tiles tuned once, then a kernel trace of
# 20 two-lane steps replaying them (no tuner dispatches in the trace), plus the per-layer table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 200 python $R/scripts/r50_profile.py --batch 320 --tune $R/gpurun_out/tiles_b320.json > $R/gpurun_out/r50_tune.log 2>&1 || { tail -20 $R/gpurun_out/r50_tune.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run -- python3 $R/scripts/r50_profile.py --batch 320 --load $R/gpurun_out/tiles_b320.json --iters 20 --lanes 2 > $R/gpurun_out/r50p_final.log 2>&1 || { tail -20 $R/gpurun_out/r50p_final.log; exit 1; }
grep "frames/s" $R/gpurun_out/r50p_final.log
db=$(find $R/gpurun_out/prof_final -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/scripts/rocprof_summary.py "$db" > $R/gpurun_out/prof_final_summary.md 2>&1
head -12 $R/gpurun_out/prof_final_summary.md
timeout -k 10 300 python $R/scripts/model_layers.py --batch 320 > $R/gpurun_out/layers_final.txt 2>&1 || { tail -20 $R/gpurun_out/layers_final.txt; exit 1; }
tail -1 $R/gpurun_out/layers_final.txt
