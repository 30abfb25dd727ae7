#!/bin/bash
# Whisper-small encoder bench at the 14-stream default under rocprofv3 (kernel trace + stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 $R/bench.py --model whisper-small --steps 20 --warmup 5 > $R/gpurun_out/wh14_bench.log 2>&1 || { tail -20 $R/gpurun_out/wh14_bench.log; exit 1; }
tail -1 $R/gpurun_out/wh14_bench.log | cut -c1-220
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wh14 -o run -- python3 $R/bench.py --model whisper-small --steps 20 --warmup 5 > $R/gpurun_out/wh14_prof.log 2>&1 || { tail -20 $R/gpurun_out/wh14_prof.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/wh14_prof.log
db=$(find $R/gpurun_out/prof_wh14 -name "*.db" | head -1)
[ -n "$db" ] && python3 $R/scripts/rocprof_summary.py "$db" > $R/gpurun_out/prof_wh14_summary.md 2>&1
head -14 $R/gpurun_out/prof_wh14_summary.md
