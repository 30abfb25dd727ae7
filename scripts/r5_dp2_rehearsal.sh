#!/bin/bash
# Rehearse the driver's N > 1 bench launch on ONE GPU: two ranks (torchrun, 127.0.0.1), both on
# cuda:0, gloo for the barrier / max-reduce (RCCL refuses two ranks on one device).  Checks the
# multi-rank bench path end to end (rank setup, barrier bracket, max over ranks, one JSON line);
# the number is two processes sharing one GPU, not a scaling point.
cd $GRAFT_REPO_ROOT
export AIKO_GPU_COMM_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
  bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/dp2.log 2>&1 || { tail -30 gpurun_out/dp2.log; exit 1; }
grep '"metric"' gpurun_out/dp2.log | cut -c1-400
