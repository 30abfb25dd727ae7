"""Stage-3 chain (conv_chain3.hip) vs the two unchained 1x1 convs, ResNet-50 B=160 / 320 shapes."""
import torch
from aiko_services_amd import ops
from aiko_services_amd.ops import conv as C

ops.require_native()
g = torch.Generator().manual_seed(0)
spec3 = C.make_conv_spec(torch.randn(1024, 256, 1, 1, generator=g) / 16, 0.1 * torch.randn(1024, generator=g),
                         act="relu", device="cuda")
spec1 = C.make_conv_spec(torch.randn(256, 1024, 1, 1, generator=g) / 32, 0.1 * torch.randn(256, generator=g),
                         act="relu", device="cuda")


def bench(fn, n=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


import os
os.environ["AIKO_CHAIN3"] = "1"
for B in (160, 320):
    x = torch.randn(B, 14, 14, 256, generator=g).to("cuda", torch.bfloat16)
    r = torch.randn(B, 14, 14, 1024, generator=g).to("cuda", torch.bfloat16)
    y = torch.empty(B, 14, 14, 1024, dtype=torch.bfloat16, device="cuda")
    z = torch.empty(B, 14, 14, 256, dtype=torch.bfloat16, device="cuda")
    y2 = torch.empty_like(y)
    z2 = torch.empty_like(z)
    C.conv_chain(x, spec3, r, y, spec1, z)
    C.conv2d(x, spec3, residual=r, out=y2)
    C.conv2d(y2, spec1, out=z2)
    dz = ((z.float() - z2.float()).norm() / z2.float().norm()).item()
    dy = ((y.float() - y2.float()).norm() / y2.float().norm()).item()
    t_chain = bench(lambda: C.conv_chain(x, spec3, r, y, spec1, z))
    t_a = bench(lambda: C.conv2d(x, spec3, residual=r, out=y2))
    t_b = bench(lambda: C.conv2d(y2, spec1, out=z2))
    M = B * 196
    mb = (M * 256 * 2 + M * 1024 * 4 + M * 256 * 2) / 1e6
    print(f"B={B} chain {t_chain:.1f} us ({mb / t_chain:.2f} TB/s)  unchained {t_a:.1f} + {t_b:.1f} = {t_a + t_b:.1f} us  "
          f"rel err y {dy:.2e} z {dz:.2e}", flush=True)
    for grid in (128, 192, 512):
        t = bench(lambda: C.conv_chain(x, spec3, r, y, spec1, z, grid=grid))
        print(f"  grid {grid}: {t:.1f} us", flush=True)
