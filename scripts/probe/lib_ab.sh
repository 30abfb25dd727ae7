#!/bin/bash
# Same-box A/B of the in-tree library vs abtmp/old_C.so on one bench command:
#   scripts/probe/lib_ab.sh ROUNDS <bench.py args...>
R=$GRAFT_REPO_ROOT
N=$1; shift
O=$R/gpurun_out/lib_ab; mkdir -p $O
OLD=/tmp/oldrepo; rm -rf $OLD; mkdir -p $OLD
(cd $R && tar cf - --exclude=./gpurun_out --exclude=./abtmp .) | (cd $OLD && tar xf -)
cp $R/abtmp/old_C.so $OLD/aiko_services_amd/_C.so
for i in $(seq $N); do
  for d in $R $OLD; do
    n=$(basename $d); cd $d
    timeout -k 10 400 python -u bench.py "$@" > $O/b_${n}_$i.log 2>&1 || { tail -5 $O/b_${n}_$i.log; exit 1; }
    echo "$n: $(grep -o '"value": [0-9.]*' $O/b_${n}_$i.log)"
  done
done
