#!/usr/bin/env python3
"""conv3x3_patchw (ResNet stage 2 3x3) isolated at batch B: mean us per launch over --iters."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=640)
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
from aiko_services_amd.ops import conv as C  # noqa: E402
from aiko_services_amd.ops import require_native  # noqa: E402
require_native()
g = torch.Generator().manual_seed(0)
w = torch.randn(128, 128, 3, 3, generator=g) / (128 * 9) ** 0.5
spec = C.make_conv_spec(w, torch.randn(128, generator=g) * 0.1, stride=1, pad=1, act="relu", device="cuda")
x = torch.randn(a.batch, 28, 28, 128, device="cuda").to(torch.bfloat16)
y = torch.empty_like(x)
wi = C.patchw_weight(spec)
f = lambda: torch.ops.aiko.conv3x3_patchw_out(x, wi, spec.bias, y, spec.act, 0)  # noqa: E731
for _ in range(5):
    f()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    f()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) / a.iters * 1e3
flop = 2 * a.batch * 784 * 128 * 1152
print(f"{us:.1f} us/launch, {flop / us / 1e9:.3f} PFLOP/s")
