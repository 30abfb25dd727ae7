#!/bin/bash
# YOLOv8-n steady-state kernel sequence: one lane (isolated per-kernel times, one forward in launch
# order) and the two-lane bench's last third of dispatches (no tuning in the summary)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5yseq; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 bench.py --model yolov8n --lanes 1 --steps 10 --warmup 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/p1 -name "*.db" | head -1) --sequence 80 > $O/seq_l1.md
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p2 -o run -- python3 bench.py --model yolov8n --steps 30 --warmup 6 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/p2 -name "*.db" | head -1) --last-frac 0.33 > $O/sum_l2.md
rm -rf $O/p1 $O/p2
tail -3 $O/seq_l1.md; head -25 $O/sum_l2.md
