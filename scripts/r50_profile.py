#!/usr/bin/env python3
"""Steady-state ResNet-50 forwards for kernel traces (no tuner launches in the trace).

    python scripts/r50_profile.py --tune gpurun_out/tiles.json          # tune, save the choices
    rocprofv3 --kernel-trace --stats -d DIR -o run -- \\
        python3 scripts/r50_profile.py --load gpurun_out/tiles.json --iters 20 --lanes 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tune", default=None, help="autotune and save the tile cache here")
    ap.add_argument("--load", default=None, help="tile cache to replay")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lanes", type=int, default=2)
    a = ap.parse_args()
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    m = ResNet50(device="cuda")
    frames = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device="cuda")
    if a.tune:
        with C.autotune():
            m.logits(frames)
        C.save_tile_cache(a.tune)
        print("tuned", len(C.tile_cache()), "geometries ->", a.tune)
        return
    if a.load:
        print("loaded", C.load_tile_cache(a.load), "geometries")
    x = torch.stack([frames, frames]) if a.lanes > 1 else frames
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for i in range(a.iters + 2):
        if i == 2:
            e0.record()
        if a.lanes > 1:
            m.logits_lanes(x.view(-1, *frames.shape[1:]), a.lanes, frames=True)
        else:
            m.logits(frames)
    e1.record()
    e1.synchronize()
    per = e0.elapsed_time(e1) / a.iters
    imgs = a.batch * (a.lanes if a.lanes > 1 else 1)
    print(f"{per:.3f} ms per {imgs}-frame step ({imgs / per * 1e3:.0f} frames/s, eager, lanes={a.lanes})")


if __name__ == "__main__":
    main()
