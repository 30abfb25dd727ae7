#!/usr/bin/env python3
"""Time single ResNet-50 conv layers (B=256) on the igemm kernel for every tile / prefetch depth.

    python scripts/layer_bench.py [--layers b0.conv3,b1.conv1] [--iters 20] [--out f.json]
Used under rocprofv3 --pmc to read counters per layer/tile (one dispatch name per variant).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

# name: (cin, cout, k, stride, hin, residual, fused_shortcut_cin)
LAYERS = {
    "b0.conv1": (64, 64, 1, 1, 56, False, 0),
    "b0.conv2": (64, 64, 3, 1, 56, False, 0),
    "b0.conv3f": (64, 256, 1, 1, 56, False, 64),
    "b1.conv1": (256, 64, 1, 1, 56, False, 0),
    "b1.conv3": (64, 256, 1, 1, 56, True, 0),
    "b3.conv1": (256, 128, 1, 1, 56, False, 0),
    "b3.conv2": (128, 128, 3, 2, 56, False, 0),
    "b4.conv2": (128, 128, 3, 1, 28, False, 0),
    "b4.conv3": (128, 512, 1, 1, 28, True, 0),
    "b8.conv2": (256, 256, 3, 1, 14, False, 0),
    "b8.conv3": (256, 1024, 1, 1, 14, True, 0),
    "b14.conv3": (512, 2048, 1, 1, 7, True, 0),
    "b14.conv2": (512, 512, 3, 1, 7, False, 0),
    "b9.conv1": (1024, 256, 1, 1, 14, False, 0),       # stage-3 reduction
    "b3.conv3f": (128, 512, 1, 1, 28, False, 256),     # stage-2 fused projection (K = 128 + 256)
    "b13.conv1": (1024, 512, 1, 1, 14, False, 0),
    "gemm4k": (4096, 4096, 1, 1, 16, False, 0),       # M = 256*16*16 = 65536: main-loop ceiling
    "gemm4k_3x3": (512, 4096, 3, 1, 16, False, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default=",".join(LAYERS))
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--tile", default=None, help="only this tile, e.g. 128,128,1")
    a = ap.parse_args()
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    dev = "cuda"
    res = {}
    for name in a.layers.split(","):
        cin, cout, k, s, hin, has_res, sc = LAYERS[name]
        g = torch.Generator().manual_seed(0)
        w = torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5
        spec = C.make_conv_spec(w, torch.zeros(cout), stride=s, pad=k // 2, act="relu", device=dev)
        x = torch.randn(a.batch, hin, hin, cin, device=dev).to(torch.bfloat16)
        x2 = None
        if sc:
            down = C.make_conv_spec(torch.randn(cout, sc, 1, 1, generator=g) / sc ** 0.5, torch.zeros(cout),
                                    device=dev)
            spec = C.fuse_shortcut(spec, down)
            x2 = torch.randn(a.batch, hin, hin, sc, device=dev).to(torch.bfloat16)
        Ho, Wo = spec.out_hw(hin, hin)
        r = torch.randn(a.batch, Ho, Wo, cout, device=dev).to(torch.bfloat16) if has_res else None
        out = torch.empty(a.batch, Ho, Wo, cout, device=dev, dtype=torch.bfloat16)
        M = a.batch * Ho * Wo
        flops = 2 * M * cout * (cin * k * k + sc)
        nbytes = (x.numel() + out.numel() + (r.numel() if r is not None else 0) + (x2.numel() if x2 is not None else 0)) * 2
        base = C.NARROW_TILES if cout <= 32 else C.TILES
        res[name] = {}
        cands = [tt + (0,) for tt in base] + ([tt + (1,) for tt in base] if cout > 32 else [])
        if cout > 32 and C.buf_variant_ok(spec, x, x2):
            cands += [tt + (2,) for tt in base + C.BUF_WIDE_TILES] + [tt + (3,) for tt in C.BUF_OCC_TILES]
            cands += [tt + (4,) for tt in C.PERSIST_TILES]
            cands += [tt + (5,) for tt in C.MF32_TILES]
        if a.tile:
            cands = [tuple(int(v) for v in a.tile.split(","))]
        for t in cands:
            for _ in range(3):
                C.conv2d(x, spec, residual=r, out=out, tile=t, x2=x2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                C.conv2d(x, spec, residual=r, out=out, tile=t, x2=x2)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            res[name][str(t)] = {"us": round(us, 2), "tflops": round(flops / us / 1e6, 1),
                                 "tbps": round(nbytes / us / 1e6, 2)}
        best = min(res[name].items(), key=lambda kv: kv[1]["us"])
        print(f"{name:10s} M={M:7d} N={cout:4d} K={spec.K:5d}  best {best[0]} {best[1]}", flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
