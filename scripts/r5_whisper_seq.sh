#!/bin/bash
# Whisper-small: one-lane kernel sequence (isolated per-kernel times of one encoder step)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5wseq; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 bench.py --model whisper-small --lanes 1 --steps 6 --warmup 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/p1 -name "*.db" | head -1) --sequence 140 > $O/seq_l1.md
python3 scripts/rocprof_summary.py $(find $O/p1 -name "*.db" | head -1) --last-frac 0.4 > $O/sum_l1.md
rm -rf $O/p1
head -24 $O/sum_l1.md
