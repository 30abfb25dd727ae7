#!/bin/bash
# bneck_fused schedule modes re-measured with the counted waits restored (B=640, isolated + bench)
R=$GRAFT_REPO_ROOT; cd $R
for m in 0 1024 2048 512 1536 2560; do
  echo -n "mode $m: "; AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 | tr '\n' ' ' || exit 1
  AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 --dual || exit 1
done
AIKO_BN_MODE=1024 timeout -k 10 60 python scripts/bneck_run.py --batch 640 --stamps | tail -1 || exit 1
AIKO_BN_MODE=2048 timeout -k 10 60 python scripts/bneck_run.py --batch 640 --stamps | tail -1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_split_t0.log 2>&1 || exit 1
AIKO_BN_MODE=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_split_t1.log 2>&1 || { tail gpurun_out/bn_split_t1.log; exit 1; }
AIKO_BN_MODE=2048 timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_split_t2.log 2>&1 || { tail gpurun_out/bn_split_t2.log; exit 1; }
echo tests ok
bash scripts/ab_multi.sh 2 - AIKO_BN_MODE=1024 AIKO_BN_MODE=2048
