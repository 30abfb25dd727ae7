"""Plain PyTorch fp32 references of the native ops — used ONLY by tests / numerics checks.

Every HIP kernel in ``csrc/kernels`` has a counterpart here operating on NCHW fp32 tensors
(torch's native layout) so the tests compare two independent implementations.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .conv import ACT_GELU, ACT_RELU, ACT_SILU, ConvSpec
from .vision import IMAGENET_MEAN, IMAGENET_STD


def act_ref(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(x)
    if act == ACT_SILU:
        return F.silu(x)
    if act == ACT_GELU:
        return F.gelu(x)
    return x


def conv_ref(x_nchw: torch.Tensor, spec: ConvSpec, residual_nchw: torch.Tensor | None = None,
             residual_after_act: bool = False) -> torch.Tensor:
    w = spec.ref_weight.to(x_nchw.device)
    b = None if spec.ref_bias is None else spec.ref_bias.to(x_nchw.device)
    if spec.kind == "stem":
        y = F.conv2d(x_nchw, w, b, stride=spec.stride, padding=spec.stem_pad)
    else:
        y = F.conv2d(x_nchw, w, b, stride=spec.stride, padding=spec.pad)
    if residual_nchw is not None and residual_after_act:
        return act_ref(y, spec.act) + residual_nchw
    if residual_nchw is not None:
        y = y + residual_nchw
    return act_ref(y, spec.act)


def linear_ref(x: torch.Tensor, spec: ConvSpec) -> torch.Tensor:
    w = spec.ref_weight.to(x.device).reshape(spec.cout, -1)
    b = None if spec.ref_bias is None else spec.ref_bias.to(x.device)
    return act_ref(F.linear(x, w, b), spec.act)


def preprocess_ref(frames_u8: torch.Tensor, size=(224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD,
                   bgr: bool = False) -> torch.Tensor:
    """uint8 NHWC -> fp32 NCHW normalised (bilinear, half-pixel centres)."""
    x = frames_u8.permute(0, 3, 1, 2).float()
    if bgr:
        x = x.flip(1)
    if tuple(x.shape[-2:]) != tuple(size):
        x = F.interpolate(x, size=size, mode="bilinear", align_corners=False)
    m = torch.tensor(mean, device=x.device).view(1, 3, 1, 1)
    s = torch.tensor(std, device=x.device).view(1, 3, 1, 1)
    return (x / 255.0 - m) / s


def nhwc_to_nchw(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 3, 1, 2).float()


def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


# ---- detection ------------------------------------------------------------------------------

def yolo_decode_ref(feats_nchw, strides, nc: int, reg_max: int = 16):
    """Per-level head outputs (fp32 NCHW, 4*reg_max + nc channels) -> boxes [B, A, 4] xyxy,
    max-class sigmoid scores [B, A], class ids [B, A] (levels concatenated, row-major)."""
    boxes, scores, classes = [], [], []
    for f, s in zip(feats_nchw, strides):
        B, _, H, W = f.shape
        f = f.float()
        box = f[:, :4 * reg_max].reshape(B, 4, reg_max, H * W).softmax(2)
        dist = (box * torch.arange(reg_max, device=f.device, dtype=torch.float32).view(1, 1, -1, 1)).sum(2)
        ys, xs = torch.meshgrid(torch.arange(H, device=f.device), torch.arange(W, device=f.device),
                                indexing="ij")
        ax = (xs.reshape(-1).float() + 0.5)
        ay = (ys.reshape(-1).float() + 0.5)
        xyxy = torch.stack([ax - dist[:, 0], ay - dist[:, 1], ax + dist[:, 2], ay + dist[:, 3]], -1) * s
        logit, c = f[:, 4 * reg_max:].reshape(B, nc, H * W).max(1)
        boxes.append(xyxy)
        scores.append(torch.sigmoid(logit))
        classes.append(c.int())
    return torch.cat(boxes, 1), torch.cat(scores, 1), torch.cat(classes, 1)


def box_iou_ref(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    iw = (torch.minimum(a[:, None, 2], b[None, :, 2]) - torch.maximum(a[:, None, 0], b[None, :, 0])).clamp(min=0)
    ih = (torch.minimum(a[:, None, 3], b[None, :, 3]) - torch.maximum(a[:, None, 1], b[None, :, 1])).clamp(min=0)
    inter = iw * ih
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    return inter / (area_a[:, None] + area_b[None, :] - inter)


def nms_ref(boxes, scores, cls, conf=0.25, iou=0.7, max_candidates=1024, max_det=300,
            max_wh=7680.0):
    """Greedy class-aware NMS for ONE image (Ultralytics ``non_max_suppression`` semantics with
    a candidate cap; ties in score -> lower anchor index first).  Returns kept anchor indices."""
    idx = torch.nonzero(scores > conf).flatten()
    if idx.numel() == 0:
        return idx
    order = torch.sort(scores[idx], descending=True, stable=True).indices
    idx = idx[order][:max_candidates]
    b = boxes[idx] + cls[idx].float()[:, None] * max_wh
    m = box_iou_ref(b, b) > iou
    removed = torch.zeros(idx.numel(), dtype=torch.bool, device=boxes.device)
    keep = []
    m = m.cpu()
    removed = removed.cpu()
    for i in range(idx.numel()):
        if removed[i]:
            continue
        keep.append(i)
        if len(keep) == max_det:
            break
        removed |= m[i] & (torch.arange(idx.numel()) > i)
    return idx[torch.tensor(keep, dtype=torch.long, device=boxes.device)]
