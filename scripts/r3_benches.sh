#!/bin/bash
# round-3 bench set on one GPU: configs 2, 4, 5 and the config-3 actor pipeline at world 1
cd $GRAFT_REPO_ROOT
run() { local tag=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/r3b_$tag.log 2>&1 || { tail -5 gpurun_out/r3b_$tag.log; exit 1; }
        echo "$tag: $(grep -o '"value": [0-9.]*' gpurun_out/r3b_$tag.log) $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/r3b_$tag.log)"; }
run resnet --steps 30 --warmup 6
run yolo --model yolov8n --steps 30 --warmup 6
run whisper --model whisper-small --steps 20 --warmup 5
run pp1 --parallel pp --steps 20 --warmup 5
