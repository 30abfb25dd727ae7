#!/bin/bash
# Same-box A/B: bneck_fused with marks in scratch (old library, abtmp/old_C.so) vs in one register.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/bn_ab; mkdir -p $O
OLD=/tmp/oldrepo; rm -rf $OLD; mkdir -p $OLD
(cd $R && tar cf - --exclude=./gpurun_out --exclude=./abtmp .) | (cd $OLD && tar xf -)
cp $R/abtmp/old_C.so $OLD/aiko_services_amd/_C.so
for i in 1 2 3; do
  for d in $R $OLD; do
    n=$(basename $d)
    cd $d
    echo -n "$n bneck B=640: "; timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 || exit 1
    echo -n "$n bneck B=640 dual: "; timeout -k 10 60 python scripts/bneck_run.py --time --iters 20 --batch 640 --dual || exit 1
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b_${n}_$i.log 2>&1 || { tail -5 $O/b_${n}_$i.log; exit 1; }
    echo "$n bench: $(grep -o '"value": [0-9.]*' $O/b_${n}_$i.log)"
  done
done
