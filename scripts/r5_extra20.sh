#!/bin/bash
# ResNet-50 layer table with the residual form of variant 20 admitted to tuning, and bench A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
AIKO_CONV_EXTRA=20 timeout -k 10 300 python3 -u scripts/model_layers.py --batch 320 > gpurun_out/layers_r50_x20.txt 2>&1 || { tail -5 gpurun_out/layers_r50_x20.txt; exit 1; }
grep ", 20)" gpurun_out/layers_r50_x20.txt; tail -1 gpurun_out/layers_r50_x20.txt
bash scripts/ab_multi.sh 2 - AIKO_CONV_EXTRA=20
