#!/bin/bash
# tail fusions with prefetched 1x1 weights and the transposed register-direct 1x1 epilogue:
# numerics, YOLO bench (tails on / off interleaved), one-lane kernel sequence
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_detect.py > gpurun_out/t2_test.log 2>&1 || { tail -30 gpurun_out/t2_test.log; exit 1; }
tail -1 gpurun_out/t2_test.log
for t in 1 0 1 0; do
  AIKO_HEAD_TAIL=$t timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/t2_b$t.log 2>&1 || { tail -5 gpurun_out/t2_b$t.log; exit 1; }
  echo "HEAD_TAIL=$t $(grep -o '"value": [0-9.]*' gpurun_out/t2_b$t.log)"
done
O=gpurun_out/t2seq; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/p1 -o run -- python3 bench.py --model yolov8n --lanes 1 --steps 10 --warmup 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
python3 scripts/rocprof_summary.py $(find $O/p1 -name "*.db" | head -1) --sequence 80 > $O/seq_l1.md
rm -rf $O/p1
grep "glds" $O/seq_l1.md | tail -8
