#!/usr/bin/env python3
"""Where does the strip stem kernel (u8 variant 2) differ from the tile kernel (variant 0)?"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    from aiko_services_amd.ops import vision as V
    require_native()
    g = torch.Generator().manual_seed(11)
    frames = torch.randint(0, 256, (2, 224, 224, 3), generator=g, dtype=torch.uint8).cuda()
    spec = C.make_stem_spec(torch.randn(64, 3, 7, 7, generator=g) / 12, torch.randn(64, generator=g) * 0.1,
                            act="relu", device="cuda")
    a = C.stem_pool_u8(frames, spec, V.IMAGENET_MEAN, V.IMAGENET_STD, variant=0)
    b = C.stem_pool_u8(frames, spec, V.IMAGENET_MEAN, V.IMAGENET_STD, variant=2)
    torch.cuda.synchronize()
    d = (a.float() - b.float()).abs() > 0
    print("mismatch fraction", d.float().mean().item())
    print("by row  ", d.any(3).any(2).any(0).int().tolist())
    print("by col  ", d.any(3).any(1).any(0).int().tolist())
    print("by chan ", d.any(2).any(1).any(0).int().tolist())
    print("by img  ", d.flatten(1).any(1).int().tolist())
    print("a[0,:3,:3,0]", a[0, :3, :3, 0].tolist(), "b", b[0, :3, :3, 0].tolist())
    print("a[0,8:11,:3,0]", a[0, 8:11, :3, 0].tolist(), "b", b[0, 8:11, :3, 0].tolist())


if __name__ == "__main__":
    main()
