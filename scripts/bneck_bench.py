#!/usr/bin/env python3
"""ResNet-50 stage 1 at batch B: the fused bottleneck kernel (bneck_fused.hip) against the
round-3 path (igemm conv1 + conv3x3_patch + conv_chain), and the whole forward both ways.

    python scripts/bneck_bench.py [--batch 320] [--th 14]
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
    ap.add_argument("--batch", type=int, default=320)
    ap.add_argument("--grid", type=str, default="0", help="workgroup counts to try (0: one per CU)")
    a = ap.parse_args()
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    B = a.batch
    m = ResNet50(device="cuda")
    frames = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
    with C.autotune():
        m.bneck = False
        m.logits(frames)
        m.bneck = True
        m.logits(frames)
    pool = torch.relu(torch.randn(B, 56, 56, 64, device="cuda")).to(torch.bfloat16)
    blk = m.blocks

    def stage1_old():
        m.bneck = False
        x, t1 = pool, None
        for bi in range(3):
            x, t1 = m._block(bi, x, "", B, 0, B, t1, chain=True)
        return x, t1

    def stage1_new(grid):
        x = pool
        outs = [m._buf("xa", (B, 56, 56, 256)), m._buf("xb", (B, 56, 56, 256))]
        for bi in range(3):
            conv3 = blk[bi].fused if blk[bi].fused is not None else blk[bi].conv3
            x = C.bneck_fused(x, blk[bi].conv1, blk[bi].conv2, conv3, out=outs[bi % 2], grid=grid)
        return x

    t_old = timeit(stage1_old)
    y_old = stage1_old()[0].clone()
    # the round-3 path also produced the stage-2 entry conv1 (chained); time it separately
    t_c1 = timeit(lambda: C.conv2d(y_old, blk[3].conv1, out=m._buf("t1x", (B, 56, 56, 128))))
    for grid in (int(t) for t in a.grid.split(",")):
        t_new = timeit(lambda: stage1_new(grid))
        y_new = stage1_new(grid)
        err = ((y_new.float() - y_old.float()).norm() / y_old.float().norm()).item()
        per = [timeit(lambda bi=bi: C.bneck_fused(pool if bi == 0 else y_old, blk[bi].conv1, blk[bi].conv2,
                                                   blk[bi].fused if blk[bi].fused is not None else blk[bi].conv3,
                                                   out=m._buf("xq", (B, 56, 56, 256)), grid=grid)) for bi in range(3)]
        nbytes = [B * 56 * 56 * 2 * (64 + 256), B * 56 * 56 * 2 * 512, B * 56 * 56 * 2 * 512]
        print(f"B={B} grid={grid}: stage 1 fused {t_new:.1f} us (blocks " +
              ", ".join(f"{t:.1f} us {nb / t / 1e6:.2f} TB/s" for t, nb in zip(per, nbytes)) +
              f") | round-3 path {t_old:.1f} us (+ stage-2 conv1 {t_c1:.1f} us unchained) | rel diff {err:.2e}")
    for flag in (False, True):
        m.bneck = flag
        t = timeit(lambda: m.logits(frames), 10)
        print(f"whole forward bneck={flag}: {t:.1f} us = {B / t * 1e6:.0f} frames/s (one lane, eager)")


if __name__ == "__main__":
    main()
