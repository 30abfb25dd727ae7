#!/usr/bin/env python3
"""Per-layer time of a model forward with the tuner's chosen kernels (B frames).

    python scripts/model_layers.py [--model resnet50|yolov8n] [--batch 256]
Records every conv2d call of one forward, then replays each alone (20 iterations) and prints
layer, GEMM shape, tile/variant, us, TFLOP/s and TB/s (input + output + residual + fused-shortcut
source bytes, each counted once; round 3's tables left the residual out), plus the sum vs the whole
forward.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    dev = "cuda"
    if a.model == "resnet50":
        from aiko_services_amd.models.resnet50 import ResNet50
        m = ResNet50(device=dev)
        frames = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device=dev)
        fwd = lambda: m.logits(frames)  # noqa: E731
    else:
        from aiko_services_amd.models.yolov8 import YOLOv8
        m = YOLOv8(scale="n", device=dev)
        frames = torch.randint(0, 256, (a.batch, 480, 640, 3), dtype=torch.uint8, device=dev)
        fwd = lambda: m.detect(frames)  # noqa: E731
    with C.autotune():
        fwd()
    calls = []
    orig = C.conv2d

    def rec(x, spec, *args, **kw):
        out = orig(x, spec, *args, **kw)
        res = kw.get("residual", args[0] if args else None)
        x2 = kw.get("x2")
        # bytes each call moves at least once: input, output, residual, and the fused shortcut's
        # second source (K - K1 channels per output pixel)
        extra = (res.numel() if res is not None else 0) + (out.shape[0] * out.shape[1] * out.shape[2] * (spec.K - spec.K1)
                                                          if x2 is not None and spec.K1 else 0)
        calls.append((spec, x.shape, out.shape, lambda: orig(x, spec, *args, **kw), extra))
        return out
    C.conv2d = rec
    import aiko_services_amd.models.resnet50 as R
    import aiko_services_amd.models.yolov8 as Y
    R.C.conv2d = rec
    Y.C.conv2d = rec
    fwd()
    C.conv2d = R.C.conv2d = Y.C.conv2d = orig
    torch.cuda.synchronize()

    def timeit(fn, n):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    total_fwd = timeit(fwd, a.iters)
    rows, tot = [], 0.0
    for i, (spec, xs, ys, fn, extra) in enumerate(calls):
        us = timeit(fn, a.iters)
        tot += us
        M = ys[0] * ys[1] * ys[2]
        flops = 2 * M * spec.cout * spec.K
        nbytes = (xs[0] * xs[1] * xs[2] * min(xs[3], spec.Cc) + M * spec.cout + extra) * 2
        key = [k for k in C._tile_cache if k[0] == M and k[1] == spec.cout and k[2] == spec.K]
        tile = C._tile_cache[key[0]] if key else "?"
        rows.append((us, f"{i:3d} M={M:7d} N={spec.cout:4d} K={spec.K:5d} R={spec.R} s={spec.stride} "
                         f"tile={tile} {us:8.1f} us {flops / us / 1e6:7.1f} TF {nbytes / us / 1e6:5.2f} TB/s"))
    for _, r in rows:
        print(r)
    print(f"convs: {len(rows)} calls, {tot:.1f} us summed; whole forward {total_fwd:.1f} us")


if __name__ == "__main__":
    main()
