#!/bin/bash
# variants 18 / 19 / 20 numerics + isolated layer timings vs the current tuner picks
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -k "igemm_matches or fused_projection" --timeout 120 --timeout-method thread 2>&1 | tail -4
for L in b4.conv2 b8.conv2; do
  for t in 128,128,9 128,128,19 128,256,19 256,128,8 256,256,8 256,256,20 256,128,20; do
    echo -n "$L $t: "; timeout -k 10 120 python scripts/layer_bench.py --layers $L --batch 320 --tile $t --iters 20 2>&1 | grep -o "best.*" || echo fail
  done
done
for L in b13.conv1 b9.conv1 b3.conv3f; do
  for t in 256,256,8 256,256,20 256,128,20 128,256,20; do
    echo -n "$L $t: "; timeout -k 10 120 python scripts/layer_bench.py --layers $L --batch 320 --tile $t --iters 20 2>&1 | grep -o "best.*" || echo fail
  done
done
for L in b14.conv3 b8.conv3; do
  for t in 256,256,8 64,128,13 256,128,20 128,256,20; do
    echo -n "$L $t: "; timeout -k 10 120 python scripts/layer_bench.py --layers $L --batch 320 --tile $t --iters 20 2>&1 | grep -o "best.*" || echo fail
  done
done
