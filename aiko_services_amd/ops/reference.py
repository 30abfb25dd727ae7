"""Plain PyTorch fp32 references of the native ops — used ONLY by tests / numerics checks.

Every HIP kernel in ``csrc/kernels`` has a counterpart here operating on NCHW fp32 tensors
(torch's native layout) so the tests compare two independent implementations.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .conv import ACT_RELU, ACT_SILU, ConvSpec
from .vision import IMAGENET_MEAN, IMAGENET_STD


def act_ref(x: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(x)
    if act == ACT_SILU:
        return F.silu(x)
    return x


def conv_ref(x_nchw: torch.Tensor, spec: ConvSpec, residual_nchw: torch.Tensor | None = None) -> torch.Tensor:
    w = spec.ref_weight.to(x_nchw.device)
    b = None if spec.ref_bias is None else spec.ref_bias.to(x_nchw.device)
    if spec.kind == "stem":
        y = F.conv2d(x_nchw, w, b, stride=2, padding=3)
    else:
        y = F.conv2d(x_nchw, w, b, stride=spec.stride, padding=spec.pad)
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
