#!/bin/bash
# control-plane ceiling on the GPU box's CPUs (gloo, 8-rank shape): flat out per hop_batch, then
# paced at config 4's 8-GPU cadence (~4.1k batches/s through rank 0).  JSON lines -> gpurun_out/hop_r5/
cd $GRAFT_REPO_ROOT
O=gpurun_out/hop_r5; mkdir -p $O
for k in 1 2 4 8; do
  timeout -k 10 120 python -m aiko_services_amd.tools.hop_bench --replicas 7 --seconds 8 --hop-batch $k 2>/dev/null | tail -1 > $O/flat_b$k.json || exit 1
  echo "flat b$k: $(cut -c1-330 $O/flat_b$k.json)"
done
for k in 1 2 4; do
  timeout -k 10 120 python -m aiko_services_amd.tools.hop_bench --replicas 7 --seconds 8 --hop-batch $k --rate 4100 2>/dev/null | tail -1 > $O/paced4100_b$k.json || exit 1
  echo "paced b$k: $(cut -c1-330 $O/paced4100_b$k.json)"
done
