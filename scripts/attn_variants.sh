#!/bin/bash
for v in ${VARIANTS:-0 1 2 3 4 5 6 7 8}; do echo -n "variant $v: "; AIKO_ATTN_VARIANT=$v python scripts/op_bench.py attn 2>&1 | grep attn: || exit $?; done
