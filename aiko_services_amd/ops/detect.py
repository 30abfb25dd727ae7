"""Detection ops (``csrc/kernels/detect_ops.hip``): nearest upsample into concat slices, YOLOv8
DFL decode and the fused top-k + class-aware NMS, all NHWC / fixed-size outputs so they are
hipGraph-capturable and their results can be all-gathered over RCCL without size exchange."""
from __future__ import annotations

import torch

__all__ = ["upsample2x", "yolo_decode", "topk_nms", "MAX_WH"]

MAX_WH = 7680.0      # class offset for class-aware NMS in one pass (boxes never exceed it)


def upsample2x(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """Nearest 2x upsample of NHWC bf16 ``x`` (channel slices allowed) into ``out``."""
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty(B, 2 * H, 2 * W, C, dtype=x.dtype, device=x.device)
    torch.ops.aiko.upsample2x_out(x, out)
    return out


def yolo_decode(feats, strides, nc: int, boxes=None, scores=None, cls=None, reg_max: int = 16):
    """Per-level head outputs ``[B, H, W, 4*reg_max + nc]`` -> boxes ``[B, A, 4]`` (xyxy,
    letterbox pixels), max-class sigmoid scores ``[B, A]``, class ids ``[B, A]``."""
    B = feats[0].shape[0]
    A = sum(f.shape[1] * f.shape[2] for f in feats)
    dev = feats[0].device
    if boxes is None:
        boxes = torch.empty(B, A, 4, dtype=torch.float32, device=dev)
    if scores is None:
        scores = torch.empty(B, A, dtype=torch.float32, device=dev)
    if cls is None:
        cls = torch.empty(B, A, dtype=torch.int32, device=dev)
    torch.ops.aiko.yolo_decode_out(list(feats), list(strides), nc, reg_max, boxes, scores, cls)
    return boxes, scores, cls


def topk_nms(boxes, scores, cls, conf: float = 0.25, iou: float = 0.7, max_candidates: int = 1024,
             max_det: int = 300, letterbox=(1.0, 0.0, 0.0, 1e9, 1e9), det=None, count=None):
    """Fused per-image candidate selection + class-aware greedy NMS.

    ``letterbox`` = (gain, pad_l, pad_t, frame_w, frame_h) maps kept boxes back to frame pixels
    (and clips).  Returns ``det`` ``[B, max_det, 6]`` (x1, y1, x2, y2, score, class; rows past
    ``count[b]`` are zero with class -1) and ``count`` ``[B]`` int32."""
    B = scores.shape[0]
    dev = scores.device
    if det is None:
        det = torch.empty(B, max_det, 6, dtype=torch.float32, device=dev)
    if count is None:
        count = torch.empty(B, dtype=torch.int32, device=dev)
    gain, pad_l, pad_t, fw, fh = letterbox
    torch.ops.aiko.topk_nms_out(boxes, scores, cls, int(max_candidates),
                                [float(conf), float(iou), MAX_WH, float(gain), float(pad_l),
                                 float(pad_t), float(fw), float(fh)], det, count)
    return det, count
