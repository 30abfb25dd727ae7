#!/usr/bin/env python3
"""Time the fused stem + max-pool kernel variants vs the unfused conv + pool at B=256, 224x224."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    from aiko_services_amd.ops import vision as V
    require_native()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    only = sys.argv[2] if len(sys.argv) > 2 else ""      # e.g. "u8v2": time just that variant
    spec = C.make_stem_spec(torch.randn(64, 3, 7, 7) / 12, torch.randn(64) * 0.1, act="relu", device="cuda")
    frames = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
    out = torch.empty(B, 56, 56, 64, dtype=torch.bfloat16, device="cuda")
    if only.startswith("u8v"):
        from aiko_services_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD
        v = int(only[3:])
        t = timed(lambda: C.stem_pool_u8(frames, spec, IMAGENET_MEAN, IMAGENET_STD, out=out, variant=v), iters=20)
        print(f"stem_pool_u8 variant {v} {t:8.1f} us")
        return
    pre = V.preprocess_frames(frames)
    stem = torch.empty(B, 112, 112, 64, dtype=torch.bfloat16, device="cuda")
    ref = V.maxpool2d(C.conv2d(pre, spec, image_hw=(224, 224), out=stem), 3, 2, 1)
    with C.autotune():
        C.conv2d(pre, spec, image_hw=(224, 224), out=stem)
    t = timed(lambda: V.maxpool2d(C.conv2d(pre, spec, image_hw=(224, 224), out=stem), 3, 2, 1, out=out))
    print(f"unfused conv+pool   {t:8.1f} us")
    for v in (0, 1):
        C.stem_pool(pre, spec, (224, 224), out=out, variant=v)
        torch.cuda.synchronize()
        ok = torch.equal(out, ref)
        t = timed(lambda: C.stem_pool(pre, spec, (224, 224), out=out, variant=v))
        print(f"stem_pool variant {v} {t:8.1f} us  exact={ok}")
    from aiko_services_amd.ops.vision import IMAGENET_MEAN, IMAGENET_STD
    outs = {}
    for v in (0, 1, 2, 3, 4):
        outs[v] = C.stem_pool_u8(frames, spec, IMAGENET_MEAN, IMAGENET_STD, variant=v).clone()
        t = timed(lambda: C.stem_pool_u8(frames, spec, IMAGENET_MEAN, IMAGENET_STD, out=out, variant=v))
        print(f"stem_pool_u8 variant {v} {t:8.1f} us  same_as_v0={torch.equal(outs[v], outs[0])}")




def debug_phases():
    """Time variant 0 with phases cut off (bit0 no pool, bit1 no epilogue, bit2 no MFMA)."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    from aiko_services_amd.ops import vision as V
    require_native()
    spec = C.make_stem_spec(torch.randn(64, 3, 7, 7) / 12, torch.randn(64) * 0.1, act="relu", device="cuda")
    frames = torch.randint(0, 256, (256, 224, 224, 3), dtype=torch.uint8, device="cuda")
    pre = V.preprocess_frames(frames)
    out = torch.empty(256, 56, 56, 64, dtype=torch.bfloat16, device="cuda")
    for dbg in (0, 1, 3, 7):
        t = timed(lambda: C.stem_pool(pre, spec, (224, 224), out=out, variant=dbg << 4))
        print(f"dbg {dbg}: {t:8.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[2] == "phases":  # noqa: SIM114
        debug_phases()
    else:
        main()
