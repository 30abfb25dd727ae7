#!/bin/bash
# ResNet-50 at the B=320 default with the half-channel strip stem: per-layer table and a kernel
# trace of the bench itself (hipGraph, 2 lanes).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python $R/scripts/model_layers.py --batch 320 > $R/gpurun_out/layers_b320.txt 2>&1 || { tail -20 $R/gpurun_out/layers_b320.txt; exit 1; }
tail -2 $R/gpurun_out/layers_b320.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b320 -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/bench_b320_prof.log 2>&1 || { tail -20 $R/gpurun_out/bench_b320_prof.log; exit 1; }
tail -1 $R/gpurun_out/bench_b320_prof.log | cut -c1-200
f=$(find $R/gpurun_out/prof_b320 -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-5 "$f" | cut -c1-160 | head -30
db=$(find $R/gpurun_out/prof_b320 -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/scripts/rocprof_summary.py "$db" > $R/gpurun_out/prof_b320_summary.md 2>&1
exit 0
