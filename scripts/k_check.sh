#!/bin/bash
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_detect.py -x -q --timeout 120 --timeout-method thread -k "stem or yolov8n" 2>&1 | tail -1 || exit 1
echo -n "stem fast: "; timeout -k 10 60 python scripts/yolo_stem_bench.py || exit 1
TESTV="15" VARIANTS="0 15" bash scripts/attn_check.sh
