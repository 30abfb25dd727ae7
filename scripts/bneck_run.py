#!/usr/bin/env python3
"""Run the fused stage-1 bottleneck (bneck_fused.hip) alone on ResNet-50 shapes, for rocprofv3
kernel traces / PMC passes:  python scripts/bneck_run.py [--batch 320] [--iters 5] [--grid 0]
[--dual]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=320)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--dual", action="store_true", help="the projection (stage entry) block")
    ap.add_argument("--time", action="store_true", help="print the mean time per launch (events)")
    ap.add_argument("--stamps", action="store_true",
                    help="per-phase cycle breakdown from wave 0's s_memtime stamps (needs --grid)")
    a = ap.parse_args()
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    m = ResNet50(device="cuda")
    blk = m.blocks[0 if a.dual else 1]
    conv3 = blk.fused if a.dual else blk.conv3
    x = torch.relu(torch.randn(a.batch, 56, 56, 64 if a.dual else 256, device="cuda")).to(torch.bfloat16)
    y = torch.empty(a.batch, 56, 56, 256, dtype=torch.bfloat16, device="cuda")
    run = lambda: C.bneck_fused(x, blk.conv1, blk.conv2, conv3, out=y, grid=a.grid)  # noqa: E731
    run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / a.iters * 1e3
    nbytes = x.numel() * 2 + y.numel() * 2
    print(f"{us:.1f} us/launch, {nbytes / us / 1e6:.2f} TB/s" if a.time else f"ok {float(y.float().abs().mean())}")
    if a.stamps:
        G = a.grid or 256
        rows = a.batch * 56 // G
        dbg = torch.zeros(G, rows + 1, 8, dtype=torch.int32, device="cuda")
        torch.ops.aiko.bneck_fused_out(x, blk.conv1.weight, blk.conv1.bias, blk.conv2.weight, blk.conv2.bias,
                                       conv3.weight, conv3.bias, y, G, dbg)
        torch.cuda.synchronize()
        st = dbg[:, :rows].long().cpu()
        st = (st - st[..., :1]) & 0xFFFFFFFF                  # cycles since the row's first stamp
        d = st[..., 1:] - st[..., :-1]
        names = ["dma", "conv2", "dma-wait", "barrier1", "conv1", "conv3", "barrier2"]
        med = d[:, 1:].float().median(dim=0).values.median(dim=0).values      # rows after the first
        tot = float(st[:, 1:, -1].float().median())
        print("per-row cycles (median over workgroups and rows), s_memtime ticks:")
        print("  " + "  ".join(f"{n} {v:.0f}" for n, v in zip(names, med.tolist())) + f"  | row {tot:.0f}")


if __name__ == "__main__":
    main()
