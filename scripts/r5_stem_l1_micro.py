"""Isolated timing: stem_l1 fused kernel vs stem kernel + l1 conv (YOLOv8-n, B=64, 480x640)."""
import torch
from aiko_services_amd import ops
from aiko_services_amd.models.yolov8 import YOLOv8
from aiko_services_amd.ops import conv as C

ops.require_native()
m = YOLOv8("n", device="cuda")
frames = torch.randint(0, 256, (64, 480, 640, 3), dtype=torch.uint8, device="cuda")


def t(fn, n=30):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


a1 = torch.empty(64, 160, 160, 32, dtype=torch.bfloat16, device="cuda")
print(f"stem_l1 fused: {t(lambda: m.stem_l1_from_frames(frames)):.1f} us", flush=True)
print(f"stem only: {t(lambda: m.stem_from_frames(frames)):.1f} us", flush=True)
a0 = m.stem_from_frames(frames)
print(f"l1 only: {t(lambda: C.conv2d(a0, m.l1, out=a1)):.1f} us", flush=True)
