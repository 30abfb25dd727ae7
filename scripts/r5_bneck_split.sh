#!/bin/bash
# bneck_fused split conv2 schedule (AIKO_BN_MODE 1024: next row's first taps at the end of
# phase B; 2048: at its start): numerics per mode, isolated timings, bench A/B
cd $GRAFT_REPO_ROOT
for m in 1024 2048; do
  AIKO_BN_MODE=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_bneck.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
done
for i in 1 2; do for m in 0 1024 2048; do for d in "" --dual; do
  echo -n "mode $m $d: "; AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 $d 2>&1 | grep us/launch || exit 1
done; done; done
AIKO_BN_MODE=1024 timeout -k 10 60 python scripts/bneck_run.py --grid 256 --stamps || exit 1
bash scripts/ab_multi.sh 3 - AIKO_BN_MODE=1024 AIKO_BN_MODE=2048
