#!/usr/bin/env python3
"""Time the fused YOLO stem (stem_direct_kernel: letterbox + normalise + 3x3/2 conv + SiLU) on
the bench batch (B=64 480x640 uint8 -> 320x320x16 bf16), for rocprofv3 --pmc passes.

    python scripts/yolo_stem_bench.py [batch] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from aiko_services_amd.models.yolov8 import YOLOv8
    from aiko_services_amd.ops import require_native
    require_native()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    m = YOLOv8(scale="n", device="cuda")
    x = torch.randint(0, 256, (B, 480, 640, 3), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        m.stem_from_frames(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        m.stem_from_frames(x)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    out_mb = B * 320 * 320 * 16 * 2 / 1e6
    in_mb = x.numel() / 1e6
    print(f"stem_direct B={B}: {us:.1f} us  ({(in_mb + out_mb) / us:.2f} TB/s over {in_mb:.0f} MB in + {out_mb:.0f} MB out)")


if __name__ == "__main__":
    main()
