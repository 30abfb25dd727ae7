#!/bin/bash
# YOLOv8-n after the fused C2f: layer table (isolated convs, whole forward), kernel summary of the
# two-lane bench under rocprofv3, bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5yolo; mkdir -p $O
timeout -k 10 300 python3 -u scripts/model_layers.py --model yolov8n --batch 64 > $O/layers.txt 2>&1 || { tail -5 $O/layers.txt; exit 1; }
tail -1 $O/layers.txt
timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"value": [0-9.]*' $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --model yolov8n --steps 20 --warmup 5 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/prof -name "*.db" | head -1) > $O/summary.md 2>&1
head -30 $O/summary.md
rm -rf $O/prof
