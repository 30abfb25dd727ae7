#!/bin/bash
# Round-6 bench lines at the final defaults (ResNet-50 B=640 in both modes, YOLOv8-n B=192,
# Whisper-small 28 streams), two of each but pp, on one box -> gpurun_out/r6bench/bench_lines.jsonl
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6bench; mkdir -p $O; rm -f $O/bench_lines.jsonl
run() {  # name seconds args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  grep -h '^{' $O/$n.log | tail -1 >> $O/bench_lines.jsonl
  grep -o '"value": [0-9.]*' $O/$n.log
}
run resnet_a 300 --steps 20 --warmup 5
run yolo_a 300 --model yolov8n --steps 20 --warmup 5
run whisper_a 400 --model whisper-small --steps 20 --warmup 5
run pp 300 --parallel pp --steps 20 --warmup 5
run resnet_b 300 --steps 20 --warmup 5
run yolo_b 300 --model yolov8n --steps 20 --warmup 5
run whisper_b 400 --model whisper-small --steps 20 --warmup 5
