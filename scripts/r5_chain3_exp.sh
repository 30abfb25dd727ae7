#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
for e in 0 1 2 3 4 7; do
  AIKO_CHAIN3_EXP=$e timeout -k 10 120 python -u scripts/r5_chain3_exp.py >> gpurun_out/chain3_exp.log 2>&1 || exit 1
done
