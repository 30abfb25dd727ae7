#!/bin/bash
# ResNet-50 round-3 profile: per-layer table, tuned tiles, kernel traces at 2 lanes and 1 lane.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python $R/scripts/model_layers.py > $R/gpurun_out/layers_r3.txt 2>&1 || { tail -20 $R/gpurun_out/layers_r3.txt; exit 1; }
tail -3 $R/gpurun_out/layers_r3.txt
timeout -k 10 200 python $R/scripts/r50_profile.py --tune $R/gpurun_out/tiles_r3.json || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3b -o run -- python3 $R/scripts/r50_profile.py --load $R/gpurun_out/tiles_r3.json --iters 20 --lanes 2 > $R/gpurun_out/r50p_r3b.log 2>&1 || exit 1
grep "frames/s" $R/gpurun_out/r50p_r3b.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r3b1 -o run -- python3 $R/scripts/r50_profile.py --load $R/gpurun_out/tiles_r3.json --iters 20 --lanes 1 > $R/gpurun_out/r50p_r3b1.log 2>&1 || exit 1
grep "frames/s" $R/gpurun_out/r50p_r3b1.log
