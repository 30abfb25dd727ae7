#!/usr/bin/env python3
"""HBM roofline probes for the expand+residual conv shapes: torch elementwise add (2 reads + 1
write) and copy on the same tensor sizes, vs the conv with and without its residual."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    for (cin, cout, hw) in ((64, 256, 56), (128, 512, 28), (256, 1024, 14), (512, 2048, 7)):
        B = 256
        x = torch.randn(B, hw, hw, cin, device="cuda").to(torch.bfloat16)
        r = torch.randn(B, hw, hw, cout, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(r)
        spec = C.make_conv_spec(torch.randn(cout, cin, 1, 1) / cin ** 0.5, torch.zeros(cout), act="relu", device="cuda")
        nb = r.numel() * 2
        t_add = timed(lambda: torch.add(r, r, out=o))
        t_copy = timed(lambda: o.copy_(r))
        with C.autotune():
            C.conv2d(x, spec, residual=r, out=o)
            C.conv2d(x, spec, out=o)
        t_res = timed(lambda: C.conv2d(x, spec, residual=r, out=o))
        t_nores = timed(lambda: C.conv2d(x, spec, out=o))
        print(f"{cin}->{cout}@{hw}: add(2R1W) {t_add:6.1f} us {3 * nb / t_add / 1e6:5.2f} TB/s | copy {t_copy:6.1f} us "
              f"{2 * nb / t_copy / 1e6:5.2f} TB/s | conv+res {t_res:6.1f} us {(3 * nb + x.numel() * 2) / t_res / 1e6:5.2f} TB/s"
              f" | conv {t_nores:6.1f} us {(nb + x.numel() * 2) / t_nores / 1e6:5.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
