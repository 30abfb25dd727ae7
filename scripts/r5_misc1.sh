#!/bin/bash
# ResNet r5 traces, isolated Whisper GEMM / row-norm timings, row-norm legacy vs persistent A/B
cd $GRAFT_REPO_ROOT
bash scripts/r50_trace.sh 320 r5 > gpurun_out/r50trace_r5.log 2>&1 || { tail -5 gpurun_out/r50trace_r5.log; exit 1; }
cd $GRAFT_REPO_ROOT
PYTHONPATH=. timeout -k 10 300 python3 scripts/lnfold_kernels.py > gpurun_out/lnk2.log 2>&1 || exit 1
for i in 1 2; do for v in 0 1; do
  echo -n "rownorm_legacy=$v: "; AIKO_ROWNORM_LEGACY=$v timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done; done
