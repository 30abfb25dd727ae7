#!/bin/bash
# ResNet bench with tuner variants excluded (AIKO_CONV_SKIP), interleaved: does a kernel that wins
# in isolation lose under two concurrent frame lanes?
set -o pipefail
export PYTHONPATH=.
for sk in none 9 2 4 3 none 9 2 4 3 none 9 2 4 3; do
  if [ "$sk" = none ]; then unset AIKO_CONV_SKIP; else export AIKO_CONV_SKIP=$sk; fi
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/skip_$sk.log 2>&1 || { tail -5 gpurun_out/skip_$sk.log; exit 1; }
  echo "skip $sk: $(grep -o '"value": [0-9.]*' gpurun_out/skip_$sk.log)"
done
