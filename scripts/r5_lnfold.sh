#!/bin/bash
# LayerNorm folded across the Whisper GEMM pairs: kernel tests, encoder parity, bench A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_transformer.py -x -q --timeout 300 --timeout-method thread -k "rowstats or ln_producer or ln_consumer or ln_fold or whisper" 2>&1 | tail -15 || exit 1
for i in 1 2; do for v in 1 0; do
  echo -n "ln_fold=$v: "; AIKO_WHISPER_LN_FOLD=$v timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 2>&1 | grep -o '"value": [0-9.]*\|"p50_latency_ms": [0-9.]*' | tr '\n' ' ' ; echo
done; done
