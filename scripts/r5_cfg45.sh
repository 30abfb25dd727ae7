#!/bin/bash
# configs 4 and 5 bench lines + YOLO per-layer table (round 5)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5cfg; mkdir -p $O
timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > $O/yolo.log 2>&1 || { tail -5 $O/yolo.log; exit 1; }
tail -1 $O/yolo.log | cut -c1-260
timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 > $O/whisper.log 2>&1 || { tail -5 $O/whisper.log; exit 1; }
tail -1 $O/whisper.log | cut -c1-260
timeout -k 10 300 python3 -u scripts/model_layers.py --model yolov8n --batch 64 > $O/layers_yolov8n_r5.txt 2>&1 || { tail -5 $O/layers_yolov8n_r5.txt; exit 1; }
grep -E "^ (44|49|54) " $O/layers_yolov8n_r5.txt; tail -1 $O/layers_yolov8n_r5.txt
