#!/bin/bash
# Round-3 profile set: ResNet-50 PMC passes, Whisper-small kernel trace, attention PMC passes.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
bash $R/scripts/pmc_bench.sh r3 || { echo "pmc_bench failed $?"; exit 1; }
echo "pmc resnet done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_wf3 -o run -- python3 $R/bench.py --model whisper-small --steps 20 --warmup 5 > $R/gpurun_out/wf3.log 2>&1 || { tail -5 $R/gpurun_out/wf3.log; exit 1; }
tail -1 $R/gpurun_out/wf3.log
timeout -k 10 200 python3 $R/bench.py --model whisper-small --steps 20 --warmup 5 > $R/gpurun_out/wf3_noprof.log 2>&1 || exit 1
tail -1 $R/gpurun_out/wf3_noprof.log
bash $R/scripts/pmc_attn.sh > $R/gpurun_out/pmc_attn_r3.txt 2>&1 || exit 1
cat $R/gpurun_out/pmc_attn_r3.txt
