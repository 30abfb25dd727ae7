"""Timing of the top-k + NMS kernel on the YOLOv8-n bench inputs (B=64 VGA frames,
random-init weights: ~6.6k anchors above conf per image, so 1024 candidates each).

History: round 2's single kernel over the full bitmask 246 us (keys + radix select 15 us,
compaction + sort 15 us, IoU bitmask 130 us, greedy scan 86 us); rounds 3-5's three kernels
83 us; round 6's single per-class kernel (detect_ops.hip nms_fused_kernel)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from aiko_services_amd.models.yolov8 import YOLOv8  # noqa: E402
from aiko_services_amd.ops import detect as DT  # noqa: E402


def main():
    from aiko_services_amd.ops import require_native
    require_native()
    m = YOLOv8(scale="n", device="cuda")
    x = torch.randint(0, 256, (64, 480, 640, 3), dtype=torch.uint8, device="cuda")
    m.detect(x) if hasattr(m, "detect") else m(x)
    cap = {}
    orig = DT.topk_nms

    def grab(boxes, scores, cls, *a, **k):
        cap.update(boxes=boxes.clone(), scores=scores.clone(), cls=cls.clone())
        return orig(boxes, scores, cls, *a, **k)
    DT.topk_nms = grab
    m.detect(x) if hasattr(m, "detect") else m(x)
    DT.topk_nms = orig
    b, s, c = cap["boxes"], cap["scores"], cap["cls"]
    print("above conf per image:", int((s > 0.25).sum(1).float().mean()))
    top = s.topk(1024, dim=1).indices
    tc = torch.gather(c, 1, top)
    per = [torch.bincount(tc[i].long(), minlength=80) for i in range(tc.shape[0])]
    mx = torch.stack([q.max() for q in per]).float()
    nz = torch.stack([(q > 0).sum() for q in per]).float()
    print(f"classes among the 1024 candidates: {nz.mean():.1f} present, largest run {mx.mean():.0f} (min {mx.min():.0f}, max {mx.max():.0f})")
    for _ in range(3):
        det, cnt = DT.topk_nms(b, s, c)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        DT.topk_nms(b, s, c, det=det, count=cnt)
    e1.record()
    torch.cuda.synchronize()
    print(f"topk_nms B=64: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us  kept/img={cnt.float().mean():.1f}")


if __name__ == "__main__":
    main()
