#!/bin/bash
# round-5 bench lines for configs 2-5 (one box): ResNet-50 (driver shape), pp world 1, YOLOv8-n, Whisper-small
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5final; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/resnet.log 2>&1 || { tail -5 $O/resnet.log; exit 1; }
grep -o '"value": [0-9.]*' $O/resnet.log
timeout -k 10 300 python -u bench.py --parallel pp --steps 20 --warmup 5 > $O/pp.log 2>&1 || { tail -5 $O/pp.log; exit 1; }
grep -o '"value": [0-9.]*' $O/pp.log
timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > $O/yolo.log 2>&1 || { tail -5 $O/yolo.log; exit 1; }
grep -o '"value": [0-9.]*' $O/yolo.log
timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 > $O/whisper.log 2>&1 || { tail -5 $O/whisper.log; exit 1; }
grep -o '"value": [0-9.]*' $O/whisper.log
