#!/bin/bash
# bneck_fused with its DMA marks in one register (no scratch, counted vmcnt waits restored):
# numerics, isolated times at B=320 / 640, bench-shape parity, two bench lines.
cd $GRAFT_REPO_ROOT
O=gpurun_out/bn_marks; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -20 $O/test.log; exit 1; }
tail -2 $O/test.log
for b in 320 640; do
  for d in "" "--dual"; do
    echo -n "B=$b $d: "; timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch $b $d || exit 1
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_bench.py -x -q -k resnet --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -20 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench$i.log 2>&1 || { tail -5 $O/bench$i.log; exit 1; }
  tail -1 $O/bench$i.log
done
