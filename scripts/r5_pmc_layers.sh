#!/bin/bash
# PMC of the stage-2 / stage-3 3x3 convs at B=320 on their tuner tiles
cd $GRAFT_REPO_ROOT
bash scripts/pmc_cmd.sh s2_3x3_w9 conv_wide $GRAFT_REPO_ROOT/scripts/layer_bench.py --layers b4.conv2 --batch 320 --tile 128,128,9 --iters 10 > /dev/null || exit 1
bash scripts/pmc_cmd.sh s2_3x3_w8 conv_wide $GRAFT_REPO_ROOT/scripts/layer_bench.py --layers b4.conv2 --batch 320 --tile 256,128,8 --iters 10 > /dev/null || exit 1
bash scripts/pmc_cmd.sh s3_3x3_w8 conv_wide $GRAFT_REPO_ROOT/scripts/layer_bench.py --layers b8.conv2 --batch 320 --tile 256,256,8 --iters 10 > /dev/null || exit 1
for t in s2_3x3_w9 s2_3x3_w8 s3_3x3_w8; do cat gpurun_out/pmccmd_$t.txt; done
