"""Pre/post-processing and pooling ops (``csrc/kernels/vision_ops.hip``), NHWC bf16."""
from __future__ import annotations

import torch

from .conv import STEM_PAD, stem_geometry

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_frames(frames: torch.Tensor, size: tuple[int, int] = (224, 224),
                      mean=IMAGENET_MEAN, std=IMAGENET_STD, bgr: bool = False,
                      out: torch.Tensor | None = None) -> torch.Tensor:
    """uint8 ``[B, H, W, 3]`` frames -> bilinear resize to ``size`` + normalise -> the
    zero-bordered ``[B, Hp, Wp, 4]`` bf16 stem buffer (image at offset (3, 3))."""
    B = frames.shape[0]
    Ho, Wo = size
    Hp, Wp = stem_geometry(Ho, Wo)
    if out is None:
        out = torch.empty(B, Hp, Wp, 4, dtype=torch.bfloat16, device=frames.device)
    torch.ops.aiko.preprocess_out(frames, out, Ho, Wo, STEM_PAD, STEM_PAD, list(mean), list(std), bgr)
    return out


def maxpool2d(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1,
              out: torch.Tensor | None = None) -> torch.Tensor:
    B, H, W, C = x.shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    if out is None:
        out = torch.empty(B, Ho, Wo, C, dtype=x.dtype, device=x.device)
    torch.ops.aiko.maxpool_out(x, out, k, s, p)
    return out


def avgpool(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    B, H, W, C = x.shape
    if out is None:
        out = torch.empty(B, C, dtype=x.dtype, device=x.device)
    torch.ops.aiko.avgpool_out(x, out)
    return out


def softmax_topk(logits: torch.Tensor, k: int = 5, prob: torch.Tensor | None = None,
                 index: torch.Tensor | None = None) -> tuple[torch.Tensor, torch.Tensor]:
    B = logits.shape[0]
    if prob is None:
        prob = torch.empty(B, k, dtype=torch.float32, device=logits.device)
    if index is None:
        index = torch.empty(B, k, dtype=torch.int32, device=logits.device)
    torch.ops.aiko.softmax_topk_out(logits, prob, index, k)
    return prob, index
