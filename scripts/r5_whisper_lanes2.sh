#!/bin/bash
# Whisper bench: frame lanes 2 / 3 / 4, interleaved (after the tail / decode fusions)
set -o pipefail
export PYTHONPATH=.
for l in 2 3 4 2 3 4; do
  timeout -k 10 300 python -u bench.py --model whisper-small --steps 20 --warmup 5 --lanes $l > gpurun_out/wl_$l.log 2>&1 || { tail -5 gpurun_out/wl_$l.log; exit 1; }
  echo "lanes $l: $(grep -o '"value": [0-9.]*' gpurun_out/wl_$l.log) $(grep -o '"p50_latency_ms": [0-9.]*' gpurun_out/wl_$l.log)"
done
