#!/bin/bash
# strip2 stem variants: exactness tests, isolated timings, interleaved bench A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "stem_pool_fused" --timeout 120 --timeout-method thread > gpurun_out/stem2_t.log 2>&1 || { tail -30 gpurun_out/stem2_t.log; exit 1; }
tail -1 gpurun_out/stem2_t.log
for v in 2 3 4 2 3 4; do timeout -k 10 60 python scripts/stem_pool_bench.py 256 u8v$v || exit 1; done
for i in 1 2; do
  for v in 2 3 4; do
    echo -n "bench variant $v: "; AIKO_STEM_U8_VARIANT=$v timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  done
done
