"""Pre/post-processing and pooling ops (``csrc/kernels/vision_ops.hip``), NHWC bf16."""
from __future__ import annotations

import torch

from .conv import STEM_PAD, stem_geometry

YOLO_MEAN = (0.0, 0.0, 0.0)
YOLO_STD = (1.0, 1.0, 1.0)

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def preprocess_frames(frames: torch.Tensor, size: tuple[int, int] = (224, 224),
                      mean=IMAGENET_MEAN, std=IMAGENET_STD, bgr: bool = False,
                      out: torch.Tensor | None = None, stem: tuple[int, int, int] = (7, 2, STEM_PAD),
                      canvas: tuple | None = None) -> torch.Tensor:
    """uint8 ``[B, H, W, 3]`` frames -> bilinear resize to ``size`` + normalise -> the
    zero-bordered ``[B, Hp, Wp, 4]`` bf16 input of a ``stem`` = (k, stride, pad) conv.

    ``canvas`` = (Hc, Wc, off_t, off_l, fill): place the resized frame at (off_t, off_l) of an
    Hc x Wc canvas filled with colour ``fill`` (letterbox, see :func:`letterbox_geometry`);
    by default the canvas is the resized frame itself.  The canvas sits at (pad, pad)."""
    B = frames.shape[0]
    Ho, Wo = size
    k, s, p = stem
    Hc, Wc = (canvas[0], canvas[1]) if canvas else (Ho, Wo)
    Hp, Wp = stem_geometry(Hc, Wc, k, s, p)
    if out is None:
        out = torch.empty(B, Hp, Wp, 4, dtype=torch.bfloat16, device=frames.device)
    torch.ops.aiko.preprocess_out(frames, out, Ho, Wo, p, p, list(mean), list(std), bgr,
                                  [float(v) for v in canvas] if canvas else [])
    return out


def letterbox_geometry(h: int, w: int, new_shape: int | tuple[int, int] = 640):
    """Aspect-preserving resize into a ``new_shape`` canvas, centred (YOLO "letterbox",
    auto=False, scale-up allowed): returns (Ho, Wo, off_t, off_l, gain)."""
    nh, nw = (new_shape, new_shape) if isinstance(new_shape, int) else new_shape
    r = min(nh / h, nw / w)
    Wo, Ho = int(round(w * r)), int(round(h * r))
    dw, dh = (nw - Wo) / 2, (nh - Ho) / 2
    return Ho, Wo, int(round(dh - 0.1)), int(round(dw - 0.1)), r


def sppf_pool(cat: torch.Tensor, c: int, k: int = 5) -> torch.Tensor:
    """YOLOv8 SPPF pools in one kernel: channels [i*c, (i+1)*c) of the [B, H, W, 4c] concat
    buffer for i = 1, 2, 3 <- the k x k / stride-1 max pool of slice i-1 (GPU, H*W <= 2048)."""
    torch.ops.aiko.sppf_pool_(cat, c, k)
    return cat


def maxpool2d(x: torch.Tensor, k: int = 3, s: int = 2, p: int = 1,
              out: torch.Tensor | None = None) -> torch.Tensor:
    B, H, W, C = x.shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    if out is None:
        out = torch.empty(B, Ho, Wo, C, dtype=x.dtype, device=x.device)
    torch.ops.aiko.maxpool_out(x, out, k, s, p)
    return out


def mean_rows(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """``x.mean(dim=1)`` of bf16 ``[B, T, C]`` in fp32 ``[B, C]`` (HIP kernel, long T).  ``x`` may
    be a T-prefix view of a longer buffer (contiguous rows, any batch pitch)."""
    if x.stride(2) != 1 or x.stride(1) != x.shape[2]:
        x = x.contiguous()
    if out is None:
        out = torch.empty(x.shape[0], x.shape[2], dtype=torch.float32, device=x.device)
    torch.ops.aiko.mean_rows_out(x, out)
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


def resize_u8(frames: torch.Tensor, size: tuple[int, int], out: torch.Tensor | None = None) -> torch.Tensor:
    """Bilinear resize of uint8 ``[B, H, W, 3]`` frames to ``size`` = (H', W') on the GPU."""
    if frames.dim() == 3:
        return resize_u8(frames[None], size, None if out is None else out[None])[0]
    B = frames.shape[0]
    if out is None:
        out = torch.empty(B, size[0], size[1], 3, dtype=torch.uint8, device=frames.device)
    torch.ops.aiko.resize_u8_out(frames.contiguous(), out)
    return out


def batchnorm(x: torch.Tensor, scale: torch.Tensor, shift: torch.Tensor, act: int = 0,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """Standalone inference BatchNorm ``act(x * scale + shift)`` over NHWC bf16 (channel
    slices allowed); ``scale = gamma / sqrt(var + eps)``, ``shift = beta - mean * scale``."""
    if out is None:
        out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
    torch.ops.aiko.batchnorm_out(x, scale, shift, out, act)
    return out


def bn_scale_shift(gamma, beta, mean, var, eps=1e-5):
    scale = gamma / torch.sqrt(var + eps)
    return scale.float().contiguous(), (beta - mean * scale).float().contiguous()
