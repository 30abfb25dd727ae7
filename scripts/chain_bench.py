#!/usr/bin/env python3
"""Time a chained 1x1 pair (conv_chain launch) against the two unchained convs at ResNet-50 B=256.

    python scripts/chain_bench.py [--shapes 128,512,128] [--hw 28] [--batch 256]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="128,512,128")
    ap.add_argument("--hw", type=int, default=28)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    k1, n1, n2 = (int(v) for v in a.shapes.split(","))
    g = torch.Generator().manual_seed(0)
    spec3 = C.make_conv_spec(torch.randn(n1, k1, 1, 1, generator=g) / k1 ** 0.5, 0.1 * torch.randn(n1, generator=g),
                             act="relu", device="cuda")
    spec1 = C.make_conv_spec(torch.randn(n2, n1, 1, 1, generator=g) / n1 ** 0.5, 0.1 * torch.randn(n2, generator=g),
                             act="relu", device="cuda")
    B, H = a.batch, a.hw
    x = torch.randn(B, H, H, k1, device="cuda").to(torch.bfloat16)
    r = torch.randn(B, H, H, n1, device="cuda").to(torch.bfloat16)
    y = torch.empty(B, H, H, n1, dtype=torch.bfloat16, device="cuda")
    z = torch.empty(B, H, H, n2, dtype=torch.bfloat16, device="cuda")
    y2, z2 = torch.empty_like(y), torch.empty_like(z)
    with C.autotune():
        C.conv2d(x, spec3, residual=r, out=y2)
        C.conv2d(y2, spec1, out=z2)
    t_a = timeit(lambda: C.conv2d(x, spec3, residual=r, out=y2))
    t_b = timeit(lambda: C.conv2d(y2, spec1, out=z2))
    t_c = timeit(lambda: C.conv_chain(x, spec3, r, y, spec1, z))
    M = B * H * H
    nbytes = (M * k1 + 2 * M * n1 + M * n2) * 2
    err_y = ((y.float() - y2.float()).norm() / y2.float().norm()).item()
    err_z = ((z.float() - z2.float()).norm() / z2.float().norm()).item()
    print(f"chain ({k1},{n1},{n2}) M={M}: unchained {t_a:.1f} + {t_b:.1f} = {t_a + t_b:.1f} us | chained {t_c:.1f} us "
          f"({nbytes / t_c / 1e6:.2f} TB/s)  rel err y {err_y:.2e} z {err_z:.2e}")


if __name__ == "__main__":
    main()
