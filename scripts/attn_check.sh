#!/bin/bash
export TMPDIR=/tmp
for v in ${TESTV:-0}; do
  AIKO_ATTN_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 120 --timeout-method thread -k "attention or whisper" 2>&1 | tail -1 || exit 1
done
for v in ${VARIANTS:-0 10 11 12}; do
  echo -n "attn variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 60 python scripts/op_bench.py attn | grep attn: || exit 1
done
