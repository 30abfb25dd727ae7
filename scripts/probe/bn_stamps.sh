#!/bin/bash
# bneck_fused phase stamps and AIKO_BN_MODE ablations at B=640, new library vs the old one
R=$GRAFT_REPO_ROOT
OLD=/tmp/oldrepo; rm -rf $OLD; mkdir -p $OLD
(cd $R && tar cf - --exclude=./gpurun_out --exclude=./abtmp .) | (cd $OLD && tar xf -)
cp $R/abtmp/old_C.so $OLD/aiko_services_amd/_C.so
for d in $R $OLD; do
  cd $d; echo "== $(basename $d)"
  timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 --stamps || exit 1
  for m in 7 128 32 4 1; do
    echo -n "mode $m: "; AIKO_BN_MODE=$m timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 || exit 1
  done
done
