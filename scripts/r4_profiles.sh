#!/bin/bash
# End-of-round-4 profile set, one GPU call: ResNet-50 per-layer table + kernel traces (1 and 2
# lanes) + PMC passes, the Whisper-small 14-stream trace, the YOLOv8-n per-layer table.
# Outputs under gpurun_out/r4prof/ (copied into profiles/ by hand).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4prof
mkdir -p $O
echo "== resnet layers"; timeout -k 10 300 python3 $R/scripts/model_layers.py --batch 320 > $O/layers_resnet50.txt 2>&1 || { tail -5 $O/layers_resnet50.txt; exit 1; }
tail -1 $O/layers_resnet50.txt
echo "== resnet traces"; bash $R/scripts/r50_trace.sh 320 r4 || exit 1
echo "== resnet pmc"; bash $R/scripts/pmc_bench.sh r4 || exit 1
python3 $R/scripts/pmc_table.py $R/gpurun_out/pmcb_r4_* --top 16 > $O/pmc_resnet50.md 2>&1 || true
head -5 $O/pmc_resnet50.md
echo "== whisper trace"; bash $R/scripts/r3_whisper14_profile.sh || exit 1
cp $R/gpurun_out/prof_wh14_summary.md $O/whisper_summary.md 2>/dev/null
rm -rf $R/gpurun_out/prof_wh14
echo "== yolo layers"; timeout -k 10 300 python3 $R/scripts/model_layers.py --model yolov8n --batch 64 > $O/layers_yolov8n.txt 2>&1 || { tail -5 $O/layers_yolov8n.txt; exit 1; }
tail -1 $O/layers_yolov8n.txt
