#!/bin/bash
# mean_rows with 1024-thread blocks: numerics, isolated timing at the Whisper shape, Whisper bench
set -o pipefail
export PYTHONPATH=.
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops_r2.py -k mean_rows > gpurun_out/mr_test.log 2>&1 || { tail -30 gpurun_out/mr_test.log; exit 1; }
tail -1 gpurun_out/mr_test.log
timeout -k 10 120 python -u - <<'PY'
import torch
from aiko_services_amd import ops
from aiko_services_amd.ops.vision import mean_rows
ops.require_native()
for B in (7, 14):
    x = torch.randn(B, 1500, 768, device="cuda").to(torch.bfloat16)
    for _ in range(3):
        mean_rows(x)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        mean_rows(x)
    e.record(); torch.cuda.synchronize()
    print(f"mean_rows B={B}: {s.elapsed_time(e) / 50 * 1e3:.1f} us", flush=True)
PY
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --model whisper-small --steps 20 --warmup 5 > gpurun_out/mr_b.log 2>&1 || { tail -5 gpurun_out/mr_b.log; exit 1; }
  grep -o '"value": [0-9.]*' gpurun_out/mr_b.log
done
