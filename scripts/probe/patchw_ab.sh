#!/bin/bash
# conv3x3_patchw without its spill (tap-1/2 offsets on the fly) vs abtmp/old_C.so: numerics,
# isolated times at B=640, bench A/B
R=$GRAFT_REPO_ROOT; cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k patchw -x -q --timeout 120 --timeout-method thread > gpurun_out/patchw_t.log 2>&1 || { tail -20 gpurun_out/patchw_t.log; exit 1; }
tail -1 gpurun_out/patchw_t.log
OLD=/tmp/oldrepo; rm -rf $OLD; mkdir -p $OLD
(cd $R && tar cf - --exclude=./gpurun_out --exclude=./abtmp .) | (cd $OLD && tar xf -)
cp $R/abtmp/old_C.so $OLD/aiko_services_amd/_C.so
for i in 1 2 3; do
  for d in $R $OLD; do
    cd $d; echo -n "$(basename $d): "; timeout -k 10 60 python scripts/probe/patchw_time.py || exit 1
  done
done
bash $R/scripts/probe/lib_ab.sh 2 --steps 20 --warmup 5
