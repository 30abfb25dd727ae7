#!/usr/bin/env python3
"""Run one op repeatedly at Whisper-small encoder shapes (for rocprofv3 --pmc / timing).

    python scripts/op_bench.py attn|rownorm|gemm_qkv|gemm_fc1|gemm_fc2|gemm_out|fc1_gelu_mx|out_mxr|fc2_mxr
                               [--batch 16] [--iters 20] [--tile bm,bn,variant]
fc1_gelu_mx is the encoder's fc1 as run: GELU + MX-fp8 output quantisation in the epilogue.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("op")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tile", default=None)
    a = ap.parse_args()
    from aiko_services_amd.ops import require_native
    from aiko_services_amd.ops import transformer as TR
    require_native()
    dev = "cuda"
    B, T, Tp, H, d = a.batch, 1500, 1501, 12, 768
    M = B * Tp
    if a.op == "rownorm":
        x = torch.randn(M, d, device=dev).to(torch.bfloat16)
        gamma = torch.rand(d, device=dev) + 0.5
        beta = torch.randn(d, device=dev) * 0.1
        q8 = torch.empty(M, d, dtype=torch.uint8, device=dev)
        s8 = torch.empty(M, dtype=torch.float32, device=dev)
        fn = lambda: TR.rownorm(x, gamma, beta, q=q8, qs=s8)  # noqa: E731
        flops = 0
    elif a.op == "attn":
        qkv = (torch.randn(M, 3 * d, device=dev) * 1.5).to(torch.bfloat16)
        out = torch.empty(M, d, dtype=torch.bfloat16, device=dev)
        ws = TR.attention_workspace(dev) if os.environ.get("AIKO_ATTN_WS", "1") != "0" else None
        fn = lambda: TR.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], out, B, H, T, Tp, 0.125, work=ws)  # noqa: E731
        flops = 4 * B * H * T * T * 64
    else:
        K, N = {"gemm_qkv": (d, 3 * d), "gemm_fc1": (d, 4 * d), "gemm_fc2": (4 * d, d), "gemm_out": (d, d),
                "fc1_gelu_mx": (d, 4 * d), "fc1_gelu": (d, 4 * d), "fc1_mx": (d, 4 * d),
                "out_mxr": (d, d), "fc2_mxr": (4 * d, d)}[a.op]
        x = torch.randn(M, K, device=dev)
        xq, xs = TR.quantize_rows_ref(x.cpu())
        xq, xs = xq.to(dev), xs.to(dev)
        lin = TR.make_fp8_linear(torch.randn(N, K) / K ** 0.5, torch.zeros(N), dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        tile = tuple(int(v) for v in a.tile.split(",")) if a.tile else None
        if a.op in ("fc1_gelu_mx", "fc1_mx"):
            u8, usc = TR.mx_buffers(M, N, dev)
            act = TR.ACT_GELU if a.op == "fc1_gelu_mx" else TR.ACT_NONE
            fn = lambda: TR.linear_fp8(xq, xs, lin, act=act, out_mx=(u8, usc), tile=tile)  # noqa: E731
        elif a.op in ("out_mxr", "fc2_mxr"):           # MX-fp8 input + bf16 residual (encoder form)
            q8, qsc = TR.mx_quantize_ref(x.cpu())
            q8, qsc = q8.to(dev), qsc.to(dev)
            res = torch.randn(M, N, device=dev).to(torch.bfloat16)
            fn = lambda: TR.linear_fp8(q8, None, lin, out=out, residual=res, x_mx=qsc, tile=tile)  # noqa: E731
        elif a.op == "fc1_gelu":
            fn = lambda: TR.linear_fp8(xq, xs, lin, act=TR.ACT_GELU, out=out, tile=tile)  # noqa: E731
        else:
            fn = lambda: TR.linear_fp8(xq, xs, lin, out=out, tile=tile)  # noqa: E731
        flops = 2 * M * N * K
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    runs = []
    for _ in range(a.reps):                     # median of `reps` back-to-back runs of `iters`
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        e1.synchronize()
        runs.append(e0.elapsed_time(e1) / a.iters * 1e3)
    us = sorted(runs)[len(runs) // 2]
    if flops:
        print(f"{a.op}: {us:.1f} us  {flops / us / 1e6:.1f} TFLOP/s", flush=True)
    else:
        print(f"{a.op}: {us:.1f} us", flush=True)


if __name__ == "__main__":
    main()
