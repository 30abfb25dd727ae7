"""Isolated timings of the Whisper-small GEMMs at the 14-stream shape (M = 21014): the LayerNorm-
folded producer / consumer kernels (gemm_fp8_ln_out) against the plain ones plus rownorm."""
import torch

from aiko_services_amd import ops
from aiko_services_amd.ops import transformer as TR

DEV = "cuda"


def timed(fn, n=30):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[n // 2]


def main():
    ops.require_native()
    torch.manual_seed(0)
    M, d = 21014, 768
    lin = {n: TR.make_fp8_linear(torch.randn(o, i) / 20, torch.randn(o) * 0.1, DEV)
           for n, (o, i) in {"qkv": (3 * d, d), "out": (d, d), "fc1": (4 * d, d), "fc2": (d, 4 * d)}.items()}
    g, b = 1 + 0.1 * torch.randn(d), 0.1 * torch.randn(d)
    fold = {n: TR.make_ln_fp8_linear(lin[n], g, b, DEV) for n in ("qkv", "fc1")}
    gd, bd = g.to(DEV), b.to(DEV)
    x = torch.randn(M, d, device=DEV).to(torch.bfloat16)
    xq, xsc = TR.mx_buffers(M, d, DEV)
    a8, asc = TR.mx_buffers(M, d, DEV)
    u8, usc = TR.mx_buffers(M, 4 * d, DEV)
    q8 = torch.empty(M, d, dtype=torch.uint8, device=DEV)
    s8 = torch.empty(M, device=DEV)
    st = torch.zeros(3, M, 2, device=DEV)
    TR.rowstats_mx(x, xq, xsc, st)
    a8.copy_(xq); asc.copy_(xsc)
    TR.rownorm(x, gd, bd, q=q8, qs=s8)
    u8.random_(0, 100)
    usc.fill_(120)
    qkv = torch.empty(M, 3 * d, dtype=torch.bfloat16, device=DEV)
    t4 = (256, 256, 4)
    rows = [
        ("rownorm (ln1/ln2 pass)", lambda: TR.rownorm(x, gd, bd, q=q8, qs=s8)),
        ("rowstats_mx", lambda: TR.rowstats_mx(x, xq, xsc, st)),
        ("qkv plain v4", lambda: TR.linear_fp8(q8, s8, lin["qkv"], out=qkv, tile=t4)),
        ("qkv MX-A v4 (no LN)", lambda: TR.linear_fp8(xq, None, lin["qkv"], out=qkv, x_mx=xsc, tile=(256, 256, 3))),
        ("qkv LN2", lambda: TR.linear_fp8_ln(xq, xsc, fold["qkv"], st, 2, out=qkv, ln_d=d)),
        ("out-proj plain v4", lambda: TR.linear_fp8(a8, None, lin["out"], out=x, residual=x, x_mx=asc, tile=t4)),
        ("out-proj LN1", lambda: TR.linear_fp8_ln(a8, asc, lin["out"], st, 1, out=x, residual=x, out_mx=(xq, xsc))),
        ("fc1 plain v4", lambda: TR.linear_fp8(q8, s8, lin["fc1"], act=3, out_mx=(u8, usc), tile=t4)),
        ("fc1 LN2", lambda: TR.linear_fp8_ln(xq, xsc, fold["fc1"], st, 2, act=3, out_mx=(u8, usc), ln_d=d)),
        ("fc2 plain v4", lambda: TR.linear_fp8(u8, None, lin["fc2"], out=x, residual=x, x_mx=usc, tile=t4)),
        ("fc2 LN1", lambda: TR.linear_fp8_ln(u8, usc, lin["fc2"], st, 1, out=x, residual=x, out_mx=(xq, xsc))),
    ]
    for name, fn in rows:
        print(f"{name:28s} {timed(fn):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
