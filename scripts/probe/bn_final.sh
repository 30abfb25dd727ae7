#!/bin/bash
# after the bneck_fused fix: the full GPU suite, ResNet bench lines (dp x2, pp), the B=640 traces
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bnfinal; mkdir -p $O
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for n in a b; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/resnet_$n.log 2>&1 || { tail -5 $O/resnet_$n.log; exit 1; }
  grep -h '^{' $O/resnet_$n.log | tail -1 >> $O/bench_lines.jsonl
done
timeout -k 10 300 python -u bench.py --parallel pp --steps 20 --warmup 5 > $O/pp.log 2>&1 || { tail -5 $O/pp.log; exit 1; }
grep -h '^{' $O/pp.log | tail -1 >> $O/bench_lines.jsonl
grep -o '"value": [0-9.]*' $O/bench_lines.jsonl
bash scripts/r50_trace.sh 640 r6bn
