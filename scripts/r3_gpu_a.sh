#!/bin/bash
# strip stem + split-KV attention: correctness then timing
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python scripts/stem_strip_debug.py > gpurun_out/strip_dbg.txt 2>&1 || { cat gpurun_out/strip_dbg.txt; exit 1; }
cat gpurun_out/strip_dbg.txt | grep -v amdgpu.ids
timeout -k 10 120 python scripts/stem_pool_bench.py 256 > gpurun_out/strip_bench.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/strip_bench.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k stem_pool tests/test_gpu_transformer.py -k "stem_pool or attention" > gpurun_out/a_tests.txt 2>&1 || { tail -30 gpurun_out/a_tests.txt; exit 1; }
tail -2 gpurun_out/a_tests.txt
for ws in 0 1; do echo -n "attn ws=$ws: "; AIKO_ATTN_WS=$ws timeout -k 10 60 python scripts/op_bench.py attn | grep attn: || exit 1; done
