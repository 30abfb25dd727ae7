#!/bin/bash
# YOLOv8-n kernel traces at the default batch: one-lane sequence + two-lane summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/ytrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/y1 -o run -- python3 bench.py --model yolov8n --lanes 1 --steps 10 --warmup 3 > $O/y1.log 2>&1 || { tail -5 $O/y1.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/y1 -name "*.db" | head -1) --sequence 90 > $O/seq_l1.md
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/y2 -o run -- python3 bench.py --model yolov8n --steps 20 --warmup 5 > $O/y2.log 2>&1 || { tail -5 $O/y2.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/y2 -name "*.db" | head -1) --last-frac 0.4 > $O/sum_l2.md
rm -rf $O/y1 $O/y2
grep -h '"value"' $O/y1.log $O/y2.log | grep -o '"value": [0-9.]*'
