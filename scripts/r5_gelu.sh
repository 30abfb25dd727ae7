#!/bin/bash
# transcendental-free GELU in the fc1 MX-out epilogue: numerics, isolated fc1, Whisper bench
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3 || exit 1
PYTHONPATH=. timeout -k 10 300 python3 scripts/lnfold_kernels.py 2>&1 | grep -E "fc1|qkv plain" || exit 1
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
