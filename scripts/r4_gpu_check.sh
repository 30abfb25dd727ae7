#!/bin/bash
# Round-4 GPU check: the new GPU tests, then the headline bench (driver shape) default /
# host ingest / without the fused stage-1 kernel.  Output under gpurun_out/r4check/.
set -o pipefail
O=gpurun_out/r4check
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_upload.py \
  tests/test_gpu_hop_streams.py tests/test_gpu_bneck.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --ingest host > $O/bench_host.log 2>&1 || { tail -20 $O/bench_host.log; exit 1; }
tail -1 $O/bench_host.log
AIKO_RESNET_BNECK=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_nobneck.log 2>&1 || { tail -20 $O/bench_nobneck.log; exit 1; }
tail -1 $O/bench_nobneck.log
