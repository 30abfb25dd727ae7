#!/bin/bash
# Round-6 evidence on one box: bench lines for configs 2-5 (ResNet-50 driver shape x2, pp world 1,
# YOLOv8-n x2, Whisper-small x2), then the YOLOv8-n kernel traces (one-lane sequence, two-lane
# summary) and the Whisper-small two-lane summary.  Output under gpurun_out/r6final/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6final; mkdir -p $O
run() {  # name seconds args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  grep -h '^{' $O/$n.log | tail -1 >> $O/bench_lines.jsonl
  grep -o '"value": [0-9.]*' $O/$n.log
}
run resnet_a 300 --steps 20 --warmup 5
run pp 300 --parallel pp --steps 20 --warmup 5
run yolo_a 300 --model yolov8n --steps 30 --warmup 6
run whisper_a 400 --model whisper-small --steps 20 --warmup 5
run resnet_b 300 --steps 20 --warmup 5
run yolo_b 300 --model yolov8n --steps 30 --warmup 6
run whisper_b 400 --model whisper-small --steps 20 --warmup 5
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/y1 -o run -- python3 bench.py --model yolov8n --lanes 1 --steps 10 --warmup 3 > $O/y1.log 2>&1 || { tail -5 $O/y1.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/y1 -name "*.db" | head -1) --sequence 80 > $O/yolo_seq_l1.md
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/y2 -o run -- python3 bench.py --model yolov8n --steps 30 --warmup 6 > $O/y2.log 2>&1 || { tail -5 $O/y2.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/y2 -name "*.db" | head -1) --last-frac 0.33 > $O/yolo_sum_l2.md
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/w2 -o run -- python3 bench.py --model whisper-small --steps 20 --warmup 5 > $O/w2.log 2>&1 || { tail -5 $O/w2.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/w2 -name "*.db" | head -1) --last-frac 0.5 > $O/whisper_sum_l2.md
rm -rf $O/y1 $O/y2 $O/w2
grep -h '"value"' $O/y1.log $O/y2.log $O/w2.log | grep -o '"value": [0-9.]*'
