#!/bin/bash
# end-of-round check: kernel tests + driver-shaped ResNet bench x3
set -o pipefail
export PYTHONPATH=.
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/fc_test.log 2>&1 || { tail -30 gpurun_out/fc_test.log; exit 1; }
tail -1 gpurun_out/fc_test.log
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fc_b.log 2>&1 || { tail -5 gpurun_out/fc_b.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/fc_b.log
done
timeout -k 10 300 python -u bench.py --model yolov8n --steps 30 --warmup 6 > gpurun_out/fc_y.log 2>&1 || { tail -5 gpurun_out/fc_y.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/fc_y.log
timeout -k 10 300 python -u bench.py --model whisper-small --steps 20 --warmup 5 > gpurun_out/fc_w.log 2>&1 || { tail -5 gpurun_out/fc_w.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/fc_w.log
