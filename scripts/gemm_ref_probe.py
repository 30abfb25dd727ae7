#!/usr/bin/env python3
"""hipBLASLt (torch.matmul) vs our conv kernel on the ResNet 1x1 GEMM shapes (no epilogue ops)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from bw_probe import timed  # noqa: E402


def main():
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    for (M, N, K) in ((802816, 256, 64), (802816, 64, 256), (200704, 512, 128), (200704, 128, 512),
                      (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)):
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        o = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        t_bl = timed(lambda: torch.matmul(a, b.t(), out=o))
        spec = C.make_conv_spec(b.float().reshape(N, K, 1, 1), None, device="cuda")
        x = a.view(1, M, 1, K)
        oo = o.view(1, M, 1, N)
        with C.autotune():
            C.conv2d(x, spec, out=oo)
        t_us = timed(lambda: C.conv2d(x, spec, out=oo))
        fl = 2 * M * N * K
        print(f"M={M:6d} N={N:4d} K={K:4d}: hipBLASLt {t_bl:7.1f} us {fl / t_bl / 1e6:6.0f} TF | aiko {t_us:7.1f} us "
              f"{fl / t_us / 1e6:6.0f} TF", flush=True)


if __name__ == "__main__":
    main()
