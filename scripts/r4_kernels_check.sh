#!/bin/bash
# Round-4 kernel checks in one GPU call: numerics of the new kernels, then the ResNet per-layer
# tuner table + bench (scripts/pw_check.sh) and the Whisper bench with the fp8 tuner verbose.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export AIKO_PW_DUAL=${AIKO_PW_DUAL:-1} AIKO_FP8_PERSIST=${AIKO_FP8_PERSIST:-1}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_transformer.py \
  -k "fused_projection or persistent or conv_pw or mx_in_and_out" > gpurun_out/r4k_t.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r4k_t.log | head -30; tail -5 gpurun_out/r4k_t.log; exit 1; }
tail -1 gpurun_out/r4k_t.log
PW_BENCH_REPS=${PW_BENCH_REPS:-1} bash scripts/pw_check.sh || exit 1
AIKO_TUNE_VERBOSE=1 timeout -k 10 300 python -u bench.py --model whisper-small --steps 20 --warmup 5 > gpurun_out/wh_r4k.log 2>&1 || { tail -5 gpurun_out/wh_r4k.log; exit 1; }
tail -1 gpurun_out/wh_r4k.log | cut -c1-220
