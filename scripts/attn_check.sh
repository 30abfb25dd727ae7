#!/bin/bash
# Numerics (tests/test_gpu_transformer.py::test_flash_attention) and timing (op_bench) of every
# attention kernel variant: AIKO_ATTN_VARIANT is read once per process, so one run per variant.
for v in ${VARIANTS:-0 1 2 3 4 5 6 7 8}; do
  AIKO_ATTN_VARIANT=$v timeout -k 10 120 python -m pytest tests/test_gpu_transformer.py -q -k flash_attention \
    --timeout 100 --timeout-method thread 2>&1 | tail -1 | sed "s/^/variant $v tests: /" || exit 1
  echo -n "variant $v: "; AIKO_ATTN_VARIANT=$v timeout -k 10 60 python scripts/op_bench.py attn 2>&1 | grep attn: || exit 1
done
