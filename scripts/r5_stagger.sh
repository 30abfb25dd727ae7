#!/bin/bash
# Lane phase experiment: lane 1 starts the timed region AIKO_BENCH_STAGGER_US late (spin kernel).
set -o pipefail
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 60 python -u scripts/r5_sleep_cal.py > gpurun_out/stg_cal.log 2>&1 || exit 1
cpu=$(tail -1 gpurun_out/stg_cal.log | awk '{print $(NF-1)}')
export AIKO_SLEEP_CYCLES_PER_US=$cpu
for st in 0 1800 0 1800 1000 2600; do
  AIKO_BENCH_STAGGER_US=$st timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/stg_$st.log 2>&1 || exit 1
  echo "stagger $st: $(grep -o '"value": [0-9.]*' gpurun_out/stg_$st.log)" >> gpurun_out/stg_summary.log
done
