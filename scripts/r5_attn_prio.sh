#!/bin/bash
# attention: s_setprio over the MFMA clusters (variants 19 / 20) — numerics, isolated timings
# (Whisper-small shapes, B = 14) and the Whisper bench
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONPATH=.
for v in 19 20; do
  AIKO_ATTN_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread -k "attention or whisper" 2>&1 | tail -1 || exit 1
done
for i in 1 2; do for v in 0 19 20; do
  echo -n "attn variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 60 python scripts/op_bench.py attn --batch 14 | grep attn: || exit 1
done; done
for v in 0 19 0 19; do
  echo -n "bench variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
