#!/bin/bash
# Stage-3 chain: numerics test, microbench, ResNet bench with and without it.
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipeline.py -k "conv_chain" > gpurun_out/chain3_test.log 2>&1 &&
timeout -k 10 200 python -u scripts/r5_chain3.py > gpurun_out/chain3_micro.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/chain3_b0.log 2>&1 &&
AIKO_CHAIN3=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/chain3_b1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/chain3_b0b.log 2>&1 &&
AIKO_CHAIN3=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/chain3_b1b.log 2>&1
