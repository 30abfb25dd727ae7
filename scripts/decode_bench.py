#!/usr/bin/env python3
"""Time the YOLOv8 DFL decode and the SPPF pools at the bench's head shapes (B=64, 640x640: 80/40/20 levels, 144 ch):
LDS-tiled kernel vs the per-anchor kernel (AIKO_DECODE_FLAT=1), same inputs, outputs compared."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        out = fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        out = fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3, out


def main():
    from aiko_services_amd.ops import detect as DT, require_native
    require_native()
    feats = [torch.randn(64, s, s, 144, device="cuda").to(torch.bfloat16) for s in (80, 40, 20)]
    fn = lambda: DT.yolo_decode(feats, (8, 16, 32), 80)  # noqa: E731
    t_tiled, a = timed(fn)
    os.environ["AIKO_DECODE_FLAT"] = "1"
    t_flat, b = timed(fn)
    same = all(torch.equal(x, y) for x, y in zip(a, b))
    print(f"yolo_decode B=64: tiled {t_tiled:.1f} us, per-anchor {t_flat:.1f} us, identical={same}")
    from aiko_services_amd.ops import vision as V
    cat = torch.randn(64, 20, 20, 512, device="cuda").to(torch.bfloat16)
    c = 128

    def chained():
        for i in range(3):
            V.maxpool2d(cat[..., i * c:(i + 1) * c], 5, 1, 2, out=cat[..., (i + 1) * c:(i + 2) * c])
    t_chain, _ = timed(chained)
    ref = cat.clone()
    t_fused, _ = timed(lambda: V.sppf_pool(cat, c, 5))
    print(f"SPPF pools [64,20,20,4x128]: fused {t_fused:.1f} us, 3 chained maxpools {t_chain:.1f} us, "
          f"identical={torch.equal(cat, ref)}")
    up_in = torch.randn(64, 40, 40, 128, device="cuda").to(torch.bfloat16)
    up_out = torch.empty(64, 80, 80, 192, device="cuda", dtype=torch.bfloat16)
    t_up, _ = timed(lambda: DT.upsample2x(up_in, out=up_out[..., :128]))
    ok = torch.equal(up_out[..., :128], up_in.repeat_interleave(2, 1).repeat_interleave(2, 2))
    print(f"upsample2x [64,40,40,128] -> slice of [64,80,80,192]: {t_up:.1f} us, exact={ok}")


if __name__ == "__main__":
    main()
