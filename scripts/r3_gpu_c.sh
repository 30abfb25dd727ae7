#!/bin/bash
# conv_wide 32-deep ring (variant 11): correctness, per-layer timing, bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "igemm_matches_torch or fused_projection" > gpurun_out/c_tests.txt 2>&1 || { tail -30 gpurun_out/c_tests.txt; exit 1; }
tail -1 gpurun_out/c_tests.txt
timeout -k 10 300 python scripts/model_layers.py > gpurun_out/layers_c.txt 2>&1 || { tail -20 gpurun_out/layers_c.txt; exit 1; }
grep -E "tile=\([0-9]+, [0-9]+, 11\)|convs:" gpurun_out/layers_c.txt | head -40
for i in 1 2; do
  echo -n "bench default: "; timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
  echo -n "bench skip 11: "; AIKO_CONV_SKIP=11 timeout -k 10 200 python bench.py --steps 30 --warmup 6 2>&1 | grep -o '"value": [0-9.]*' || exit 1
done
