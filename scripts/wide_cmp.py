#!/usr/bin/env python3
"""Per-layer A/B of the conv kernel variants on a model's real conv calls (one GPU).

    python scripts/wide_cmp.py [--model resnet50] [--batch 256] [--variants 8] [--iters 20]
Records every conv2d call of one forward, then for each call times every candidate tile of the
older kernels (the tuner's pool without the listed variants) and of the listed variants, in one
process, interleaved, and prints the best of each side per layer and the summed totals.
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
    ap.add_argument("--variants", default="8,9,10")
    a = ap.parse_args()
    new_v = {int(v) for v in a.variants.split(",")}
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
    calls = []
    orig = C.conv2d

    def rec(x, spec, *args, **kw):
        out = orig(x, spec, *args, **kw)
        kw2 = dict(kw)
        kw2.pop("tile", None)
        calls.append((spec, x, args, kw2, out))
        return out
    import aiko_services_amd.models.resnet50 as R
    import aiko_services_amd.models.yolov8 as Y
    C.conv2d = R.C.conv2d = Y.C.conv2d = rec
    fwd()
    C.conv2d = R.C.conv2d = Y.C.conv2d = orig
    torch.cuda.synchronize()

    def timeit(fn, n):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / n * 1e3

    tot_old = tot_new = tot_best = 0.0
    for li, (spec, x, args, kw, out) in enumerate(calls):
        x2 = kw.get("x2")
        if not C.buf_variant_ok(spec, x, x2):
            continue
        cands = [t + (0,) for t in C.TILES] + [t + (1,) for t in C.TILES]
        cands += [t + (2,) for t in C.TILES + C.BUF_WIDE_TILES] + [t + (3,) for t in C.BUF_OCC_TILES]
        cands += [t + (4,) for t in C.PERSIST_TILES] + [t + (5,) for t in C.MF32_TILES]
        cands += [t + (6,) for t in C.WIDE4_TILES] + [t + (8,) for t in C.WIDE8_TILES]
        cands += [t + (9,) for t in C.WIDE_OCC_TILES]
        if C.patch_variant_ok(spec, x, kw.get("residual"), x2, out):
            cands.append((8, 64, 10))
        res = {}
        for t in cands:
            def fn(t=t):
                orig(x, spec, *args, tile=t, **kw)
            try:
                res[t] = timeit(fn, a.iters)
            except RuntimeError as e:       # unsupported tile for this shape
                print("  skip", t, str(e).splitlines()[0][:80])
        old = {t: us for t, us in res.items() if t[2] not in new_v}
        new = {t: us for t, us in res.items() if t[2] in new_v}
        bo = min(old.items(), key=lambda kv: kv[1])
        bn = min(new.items(), key=lambda kv: kv[1]) if new else (None, float("inf"))
        Ho, Wo = out.shape[1], out.shape[2]
        M = out.shape[0] * Ho * Wo
        flops = 2 * M * spec.cout * spec.K
        tot_old += bo[1]
        tot_new += min(bn[1], 1e9)
        tot_best += min(bo[1], bn[1])
        print(f"{li:3d} M={M:7d} N={spec.cout:4d} K={spec.K:5d} R={spec.R} s={spec.stride} res={'residual' in kw or len(args) > 0}"
              f" old {bo[0]} {bo[1]:7.1f} us {flops / bo[1] / 1e6:6.0f} TF | new {bn[0]} {bn[1]:7.1f} us"
              f" {flops / bn[1] / 1e6:6.0f} TF  x{bo[1] / bn[1]:.2f}", flush=True)
    print(f"sum old {tot_old:.1f} us  new {tot_new:.1f} us  best-of {tot_best:.1f} us")


if __name__ == "__main__":
    main()
