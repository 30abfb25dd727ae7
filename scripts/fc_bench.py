#!/usr/bin/env python3
"""ResNet-50 classifier layer (B=256, 2048 -> 1000, bf16): our igemm linear vs hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    m = ResNet50(device="cuda")
    f = torch.randn(256, 2048, device="cuda").to(torch.bfloat16)
    out = torch.empty(256, 1000, dtype=torch.bfloat16, device="cuda")
    spec = m.fc
    w = spec.weight[:, :2048].contiguous()
    bb = spec.bias.to(torch.bfloat16)
    print("weight", tuple(spec.weight.shape), "K", spec.K)
    print(f"igemm linear: {timeit(lambda: C.linear(f, spec, out=out)):.1f} us")
    print(f"addmm (hipBLASLt): {timeit(lambda: torch.addmm(bb, f, w.t(), out=out)):.1f} us")
    work = torch.empty(C.LINEAR_SPLITK * 256 * 1000, device="cuda")
    print(f"split-K linear (S={C.LINEAR_SPLITK}): {timeit(lambda: C.linear(f, spec, out=out, work=work)):.1f} us")
    ref = f.float() @ w.float().t() + spec.bias
    C.linear(f, spec, out=out)
    e1 = (out.float() - ref).abs().max().item()
    torch.addmm(bb, f, w.t(), out=out)
    e2 = (out.float() - ref).abs().max().item()
    print(f"max err igemm {e1:.4f} addmm {e2:.4f}")


if __name__ == "__main__":
    main()
