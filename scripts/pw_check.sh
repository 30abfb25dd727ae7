#!/bin/bash
# conv_pw (variants 12 / 13): numerics, then the tuner's candidates on the ResNet layers at B=320 and the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "conv_igemm_matches_torch or conv_pw" --timeout 120 --timeout-method thread > gpurun_out/pw_t.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/pw_t.log | head -30; tail -5 gpurun_out/pw_t.log; exit 1; }
tail -1 gpurun_out/pw_t.log
AIKO_TUNE_VERBOSE=1 timeout -k 10 300 python scripts/model_layers.py --batch 320 > gpurun_out/tune_pw.txt 2>&1 || { tail -20 gpurun_out/tune_pw.txt; exit 1; }
grep -E "1[23]\): " gpurun_out/tune_pw.txt | head -30
grep -E "^ +(5|6|10|11|13|16|19|29|31|34|37) M" gpurun_out/tune_pw.txt
tail -1 gpurun_out/tune_pw.txt
for i in $(seq 1 ${PW_BENCH_REPS:-2}); do
  echo -n "bench default: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  if [ -n "$PW_BENCH_AB" ]; then
    echo -n "bench skip $PW_BENCH_AB: "; AIKO_CONV_SKIP=$PW_BENCH_AB timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  fi
done
