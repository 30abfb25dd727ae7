"""Convolution / linear layers on the implicit-GEMM MFMA kernel (``csrc/kernels/conv_igemm.hip``).

Layouts (MI355X-first, chosen for the kernel, not for torch):

* activations are NHWC bf16 (``[B, H, W, C]`` contiguous) so an output pixel's channels are a
  contiguous GEMM row and every conv becomes ``[B*Ho*Wo, K] x [K, Cout]``;
* weights are packed once to ``[Cout, K]`` bf16 with K ordered (r, s, c) — the "B^T" layout
  whose rows the kernel stages into LDS exactly like the activation rows;
* BatchNorm is folded into the weights and an fp32 bias at pack time (inference), and the
  bias / residual add / ReLU|SiLU run in the kernel epilogue.

The ResNet stem (7x7/s2, 3 input channels) uses a pre-padded 4-channel input written by the
fused pre-processing kernel: with 4 channels per pixel a 32-element chunk of one input row
covers the 7 horizontal taps of one filter row, so the stem is an implicit GEMM with K = 8x32
(see :func:`make_stem_spec`).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

ACT_NONE, ACT_RELU, ACT_SILU, ACT_GELU = 0, 1, 2, 3
ACT_RESIDUAL_AFTER = 16          # epilogue flag: y = act(acc + b) + residual (CSP bottlenecks)
_ACTS = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "silu": ACT_SILU, "gelu": ACT_GELU}


@dataclass
class ConvSpec:
    """A packed, inference-ready conv (or linear) layer."""

    weight: torch.Tensor            # [Cout, K] bf16
    bias: torch.Tensor | None       # [Cout] fp32
    cin: int
    cout: int
    R: int
    S: int
    stride: int
    pad: int
    Cc: int                         # contiguous channel run per tap (multiple of 8)
    act: int = ACT_NONE
    kind: str = "conv"              # conv | stem | linear
    ref_weight: torch.Tensor | None = field(default=None, repr=False)  # fp32 OIHW (folded)
    ref_bias: torch.Tensor | None = field(default=None, repr=False)
    # second A source (fused 1x1 projection shortcut): K columns [K1, K) read x2
    K1: int | None = None
    stride2: int = 1
    # stem geometry (kind == "stem"): the real kernel size / padding over the image
    stem_k: int = 7
    stem_pad: int = 3

    def to(self, device) -> "ConvSpec":
        self.weight = self.weight.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        return self

    @property
    def K(self) -> int:
        return self.weight.shape[1]

    def out_hw(self, H: int, W: int) -> tuple[int, int]:
        if self.kind == "stem":
            return stem_out_hw(H, W, self.stem_k, self.stride, self.stem_pad)
        return ((H + 2 * self.pad - self.R) // self.stride + 1,
                (W + 2 * self.pad - self.S) // self.stride + 1)

    def flops(self, B: int, H: int, W: int) -> int:
        Ho, Wo = self.out_hw(H, W)
        k_real = self.cin * self.R * self.S if self.kind != "stem" else 3 * self.stem_k ** 2
        return 2 * B * Ho * Wo * self.cout * k_real


def _act(act) -> int:
    return act if isinstance(act, int) else _ACTS[act]


def fold_bn(w: torch.Tensor, gamma, beta, mean, var, eps=1e-5, conv_bias=None):
    """Fold inference BatchNorm into (weight, bias) — fp32."""
    scale = gamma / torch.sqrt(var + eps)
    wf = w * scale.reshape(-1, *([1] * (w.dim() - 1)))
    b = beta - mean * scale
    if conv_bias is not None:
        b = b + conv_bias * scale
    return wf, b


def make_conv_spec(w_oihw: torch.Tensor, bias: torch.Tensor | None, stride=1, pad=0, act=None,
                   device=None, cin_pitch: int | None = None) -> ConvSpec:
    """Pack an fp32 OIHW conv weight into the kernel's ``[Cout, K]`` bf16 layout.

    K is ordered (r, s, c) with the channel run padded to a multiple of 8 (``Cc``) and the
    total padded to a multiple of 64 with zero weights.  ``cin_pitch`` is the channel pitch
    of the input activation (defaults to ``Cc``).
    """
    cout, cin, R, S = w_oihw.shape
    cc = _round_up(cin, 8)
    k_real = R * S * cc
    K = _round_up(k_real, 64)
    w = torch.zeros(cout, R, S, cc, dtype=torch.float32)
    w[..., :cin] = w_oihw.permute(0, 2, 3, 1).float()
    packed = torch.zeros(cout, K, dtype=torch.float32)
    packed[:, :k_real] = w.reshape(cout, k_real)
    packed = packed.to(torch.bfloat16).contiguous()
    ref_w = w_oihw.to(torch.bfloat16).float().contiguous()
    spec = ConvSpec(weight=packed, bias=None if bias is None else bias.float().contiguous(),
                    cin=cin_pitch or cc, cout=cout, R=R, S=S, stride=stride, pad=pad, Cc=cc,
                    act=_act(act), kind="conv", ref_weight=ref_w,
                    ref_bias=None if bias is None else bias.float().clone())
    return spec.to(device) if device is not None else spec


def fuse_shortcut(main: ConvSpec, down: ConvSpec) -> ConvSpec:
    """Fuse a 1x1 projection shortcut into a block's last 1x1 conv by K-concatenation:
    ``act(main(x) + down(x2) + b_main + b_down)`` becomes ONE igemm over ``[x | x2]`` with
    weights ``[W_main | W_down]`` — the shortcut activation is never written to HBM and the
    residual is never read back."""
    assert main.R == main.S == 1 and down.R == down.S == 1 and main.cout == down.cout
    assert main.stride == 1 and down.pad == 0
    bias = None
    if main.bias is not None or down.bias is not None:
        bias = (main.bias if main.bias is not None else 0) + (down.bias if down.bias is not None else 0)
    return ConvSpec(weight=torch.cat([main.weight, down.weight], dim=1).contiguous(), bias=bias,
                    cin=main.cin, cout=main.cout, R=1, S=1, stride=1, pad=0, Cc=main.Cc, act=main.act,
                    kind="conv", K1=main.K, stride2=down.stride)


def make_linear_spec(w_oi: torch.Tensor, bias: torch.Tensor | None, act=None, device=None) -> ConvSpec:
    cout, cin = w_oi.shape
    spec = make_conv_spec(w_oi.reshape(cout, cin, 1, 1), bias, act=act, device=device)
    spec.kind = "linear"
    return spec


# ---- stems: k x k / stride s over 3 channels, on a pre-padded 4-channel input ------------------
#
# The pre-processing kernel writes the image into a zero-bordered [B, Hp, Wp, 4] bf16 buffer.
# With 4 channels per pixel a run of P pixels of one input row is 4P contiguous elements, so
# one filter row (k taps) is a single contiguous "channel run" Cc = 4P (P = k rounded up to an
# even count, keeping Cc a multiple of 8): the stem becomes an implicit GEMM with R = k filter
# rows, S = 1, pad 0 (the padding is in the buffer) and K = k * Cc.  ResNet 7x7/2: Cc = 32;
# YOLOv8 3x3/2: Cc = 16, K = 48 -> one 64-wide K block.

STEM_PAD = 3


def stem_out_hw(H: int, W: int, k: int = 7, s: int = 2, p: int = STEM_PAD) -> tuple[int, int]:
    return (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1


def _stem_pixels(k: int) -> int:
    return k + (k & 1)


def stem_geometry(H: int, W: int, k: int = 7, s: int = 2, p: int = STEM_PAD) -> tuple[int, int]:
    """(Hp, Wp) of the zero-bordered 4-channel stem input for an HxW image (image at (p, p))."""
    Ho, Wo = stem_out_hw(H, W, k, s, p)
    Hp = max(s * (Ho - 1) + k, H + 2 * p)
    Wp = _round_up(max(s * (Wo - 1) + _stem_pixels(k), W + 2 * p), 8)
    return Hp, Wp


def make_stem_spec(w_oihw: torch.Tensor, bias: torch.Tensor | None, act="relu", device=None,
                   stride: int = 2, pad: int | None = None) -> ConvSpec:
    """Pack a [Cout, 3, k, k] stem weight as k filter rows x (P pixels x 4 channels)."""
    cout, cin, R, S = w_oihw.shape
    assert cin == 3 and R == S, "stem packing expects a square conv over 3 channels"
    k = R
    P = _stem_pixels(k)
    cc = 4 * P
    K = _round_up(k * cc, 64)
    w = torch.zeros(cout, k, P, 4, dtype=torch.float32)  # [o][r][s(pixel)][c]
    w[:, :, :k, :3] = w_oihw.permute(0, 2, 3, 1).float()
    packed = torch.zeros(cout, K, dtype=torch.float32)
    packed[:, :k * cc] = w.reshape(cout, k * cc)
    packed = packed.to(torch.bfloat16).contiguous()
    ref_w = w_oihw.to(torch.bfloat16).float().contiguous()
    spec = ConvSpec(weight=packed, bias=None if bias is None else bias.float().contiguous(),
                    cin=3, cout=cout, R=k, S=1, stride=stride, pad=0, Cc=cc, act=_act(act),
                    kind="stem", ref_weight=ref_w,
                    ref_bias=None if bias is None else bias.float().clone(),
                    stem_k=k, stem_pad=(k // 2) if pad is None else pad)
    return spec.to(device) if device is not None else spec


def _round_up(v: int, m: int) -> int:
    return (v + m - 1) // m * m


TILES = ((128, 128), (128, 64), (64, 128), (64, 64))
NARROW_TILES = ((128, 32), (256, 32), (64, 64), (128, 64))   # Cout <= 32 (YOLO stems / heads)
_tile_cache: dict = {}          # geometry key -> (bm, bn), filled by autotune()
_tuning = False
_TUNE_VERBOSE = __import__("os").environ.get("AIKO_TUNE_VERBOSE", "0") == "1"
class autotune:
    """Context manager: while active, every conv whose geometry has no cached tile times each
    candidate tile on the GPU (3 runs, HIP events) and keeps the fastest — like a conv
    "benchmark mode".  Wave quantisation (tiles vs 256 CUs x 2 blocks) makes the best tile
    shape-dependent; measuring beats modelling it."""

    def __enter__(self):
        global _tuning
        self._prev = _tuning
        _tuning = True
        return self

    def __exit__(self, *exc):
        global _tuning
        _tuning = self._prev


def tile_cache() -> dict:
    return dict(_tile_cache)


def save_tile_cache(path: str) -> None:
    """Write the tuner's per-geometry choices as JSON (profiling runs replay them without
    re-tuning, so a kernel trace holds only the steady-state launches)."""
    import json
    rows = [[list(k), list(v)] for k, v in _tile_cache.items()]
    with open(path, "w") as f:
        json.dump(rows, f)


def load_tile_cache(path: str) -> int:
    """Merge a :func:`save_tile_cache` file into the tuner's cache; returns the entry count."""
    import json
    with open(path) as f:
        rows = json.load(f)
    for k, v in rows:
        _tile_cache[tuple(k)] = tuple(v)
    return len(rows)


_ZERO: dict = {}


def zero_page(device) -> torch.Tensor:
    """64 zero bytes on ``device``: the global source of conv zero padding for the LDS-DMA
    kernel variant (allocated on first use, outside any graph capture)."""
    z = _ZERO.get(device)
    if z is None:
        z = _ZERO[device] = torch.zeros(32, dtype=torch.bfloat16, device=device)
    return z


BUF_WIDE_TILES = ((256, 128), (128, 256), (256, 64))   # 8-wave buffer-DMA kernels (one workgroup per CU)
BUF_OCC_TILES = ((64, 64), (64, 128), (128, 64))       # variant 3: buffer-DMA at 5 / 3 / 3 workgroups per CU
PERSIST_TILES = ((64, 128),)   # variant 4: persistent, one K-block ring across tiles (2 workgroups/CU)
# variant 5: buffer-DMA kernel on v_mfma_f32_32x32x16_bf16 (3x the free issue slots per MFMA)
MF32_TILES = ((128, 128), (128, 64), (64, 128), (256, 128), (128, 256))
# variant 6: 4 waves of 128 x 64 / 64 x 128 per workgroup, one workgroup per CU (fewer LDS
# fragment bytes per MFMA than the 8-wave 64 x 64 layouts of BUF_WIDE_TILES).  Measured on the
# ResNet-50 layers: never the tuner's pick — one wave per SIMD exposes the DMA / LDS latency
# that the 8-wave layouts hide — kept as a candidate for other shapes
WIDE4_TILES = ((256, 128), (128, 256))
# variant 8 (conv_wide.hip): 8 waves, transposed product (weights on the MFMA A side) so each
# lane ends with 8 consecutive output channels of one pixel and the epilogue goes straight from
# registers to memory (no LDS round trip) — tiles up to 256 x 256
WIDE8_TILES = ((256, 256), (256, 128), (128, 256), (256, 64), (128, 128))
# variant 19: the same kernel with 4 waves of 64 x 64 (128 x 128 tile, 2 workgroups per CU) or
# 64 x 128 (128 x 256, one per CU): half / a third fewer fragment reads per MFMA than the 8-wave
# 128-wide forms, whose 64 x 32 wave tiles read 0.75 fragments per MFMA.  Measured at B=320
# (round 5, scripts/r5_tiles.sh): stage-2 3x3 84.4 vs 81.2 us (variant 9), stage-3 3x3 79.9 vs
# 66.0 us (variant 8) — the fragment traffic was not the limit; opt-in (AIKO_CONV_EXTRA=19)
WIDE4_OCC_TILES = ((128, 128), (128, 256))
# variant 20: persistent conv_wide (one workgroup per CU walks tiles with ONE K-block ring across
# tile boundaries; epilogue stores always issued, so the next tile's first-block wait is exact)
# for the short-K layers without a residual (reductions, projections).  Measured at B=320 (round
# 5): fused stage-2 projection 159.6 vs 163.6 us (variant 8), stage-3 reduction 37.4 vs 36.1,
# stage-3 -> 4 reduction 70.6 vs 66.1 — the tile-boundary fill was not the limit either; the
# tuner keeps it where it wins (residual form, isolated at B=320: 60-61 vs 49.7 us at stage 4,
# 87.6 vs 76.7 us at stage 3 against the resident-weight kernel)
WIDE_PERS_TILES = ((256, 256), (256, 128), (128, 256))
# variant 18: the same kernel with an exact-N tile (the MFMAs and epilogue cover exactly
# these channel counts — the YOLO head's 80-class and 64 + 80 box/class convs — instead of
# rounding N up to a 128 / 192 tile; odd 16-channel block counts end in an 8-byte store)
EXACT_N = (80, 144)
# exact-N tiles of the LDS-DMA igemm (variant 1, conv_glds.hip: 4 x 1 waves, each all N columns)
# for N = 80 layers whose 80-channel input (Cc = 80) rules out every 64-channel-block kernel: the
# YOLOv8 class branch (3x3 80 -> 80, 1x1 80 -> 80), where a 128-wide tile wastes 37.5 % of its lanes
GLDS_EXACT_N = (80,)
# variant 9: the same kernel at 2-3 workgroups per CU (short-K, bandwidth-bound layers)
WIDE_OCC_TILES = ((128, 128), (256, 64), (128, 64), (64, 128), (64, 64))
# variant 11: the same kernel with 32-deep K blocks in a 4-slot ring (three blocks in flight
# across each barrier instead of one for the 256-wide tiles) — the long-K compute-bound layers.
# Measured on the ResNet-50 layers (MI355X, round 3): never the tuner's pick against variant 8,
# i.e. the 2-slot 64-deep ring is not what limits those tiles; kept as a candidate.  Round 4: a
# 256 x 256 form with split rings (3 activation slots + 2 weight slots = 160 KB, activations two
# blocks ahead) measured 70.8 vs 68.0 us on the stage-3 3x3 (PMC of variant 11 vs 8: wait share
# 37 vs 40 %, twice the L2 requests at 64-B rows) — dropped
WIDE_DEEP_TILES = ((256, 256), (256, 128), (128, 256))
# variant 12 (conv_pw.hip): persistent pointwise GEMM for 1x1/s1 convs with K % 256 == 0 — one
# 4-slot K-block ring across tile boundaries, residual DMA'd into LDS, fixed channel block per
# workgroup; 77.9 vs 80 us on the stage-3 expansion at B=320.  Variant 13 (K == 256): the
# workgroup's 128 x 256 weight block resident in LDS, 64-pixel tiles through an 8-slot ring (seven
# blocks in flight): 65.6 us there (the tuner's pick; 500 TF, 4.4 TB/s counting the residual).
# Round 4: variant 13 also takes K == 128 (256 x 128 weight block, 4-slot ring) and DMAs the residual
# one tile ahead; variant 14 is the same kernel with the residual issued at its own tile (A/B form,
# tuned only with AIKO_PW_AB=1).  Measured at B=320 (scripts/pw_check.sh, same box): K=128 -> 512
# expansion 105.5 (13) vs 110.9 us (14) and vs 133 us for the best tiled kernel (5.6 TB/s counting the
# residual); K=256 -> 1024 71.4 vs 71.8; K=512 -> 2048 81.1 vs 79.8 (the tiled kernel, 47 us, wins)
_PW_AB = __import__("os").environ.get("AIKO_PW_AB") == "1"
# opt-in tuner variants (never picked on the measured models): AIKO_CONV_EXTRA="6,11"
_EXTRA = {int(v) for v in __import__("os").environ.get("AIKO_CONV_EXTRA", "").split(",") if v.strip().isdigit()}
# variant 13 as the fused stage-2 projection (conv_pw_rb_kernel<false, 384, 1, 128>) in the tuner:
# numerics-tested but measured slower than conv_wide's 256 x 256 tile (167 vs 154 us at B=320 — the
# strided second source streams from HBM behind a 5-block lookahead), so opt-in
_PW_DUAL = __import__("os").environ.get("AIKO_PW_DUAL", "0") == "1"


def buf_variant_ok(spec: ConvSpec, x: torch.Tensor, x2: torch.Tensor | None = None) -> bool:
    """Whether the buffer-LDS-DMA kernel (variant 2) applies: whole 64-channel K blocks per tap
    and operands addressable with 31-bit byte offsets."""
    def nbytes(t):
        return t.untyped_storage().nbytes() - t.storage_offset() * t.element_size()
    return (spec.kind != "stem" and spec.Cc % 64 == 0 and spec.R * spec.S <= 32 and spec.cout > 32
            and nbytes(x) < 2**31 - 64 and spec.weight.numel() * 2 < 2**31
            and (x2 is None or nbytes(x2) < 2**31 - 64))


def patch_variant_ok(spec: ConvSpec, x: torch.Tensor, residual=None, x2=None, out=None) -> bool:
    """Whether the LDS-resident-patch 3x3 kernel (variant 10, conv_patch.hip) applies: a 3x3 /
    stride 1 / pad 1 conv 64 -> 64 channels on a contiguous [B, H, W, 64] input (W = 56, 40 or 24:
    the kernel's patch pitch is a compile-time constant), no residual,
    no second source, activation none / ReLU / SiLU."""
    return (spec.kind == "conv" and spec.R == 3 and spec.S == 3 and spec.stride == 1 and spec.pad == 1
            and spec.Cc == 64 and spec.cout == 64 and spec.K == 576 and spec.K1 is None
            and residual is None and x2 is None and spec.act in (ACT_NONE, ACT_RELU, ACT_SILU)
            and x.dim() == 4 and x.shape[3] == 64 and x.is_contiguous() and x.shape[2] in (56, 40, 24)
            and (out is None or (out.stride(3) == 1 and out.stride(2) % 8 == 0)))


def patch_weight(spec: ConvSpec) -> torch.Tensor:
    """[9, 2, 4, 64, 8] MFMA fragment image of a 3x3 64 -> 64 weight for conv_patch.hip: (tap,
    32-channel half, 16-output-channel block, lane = 16 (k chunk) + output row, 8 channels).  Cached
    on the spec and re-derived in place when the weight changes (as stem_pool_weight)."""
    key = (spec.weight.data_ptr(), spec.weight._version)
    cached = getattr(spec, "_patch_w", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    w = spec.weight.view(4, 16, 9, 2, 4, 8)                  # [nb, fr, tap, half, fq, e]
    img = w.permute(2, 3, 0, 4, 1, 5).reshape(9, 2, 4, 64, 8)
    if cached is not None:
        cached[1].copy_(img)
        img = cached[1]
    else:
        img = img.contiguous()
    spec._patch_w = (key, img)
    return img


def patchw_variant_ok(spec: ConvSpec, x: torch.Tensor, residual=None, x2=None, out=None) -> bool:
    """Whether the streamed-weight patch 3x3 kernel (variant 16, conv_patchw.hip) applies: a 3x3 /
    stride 1 / pad 1 conv 128 -> 128 channels on an NHWC [B, H, 28, >= 128] input (the ResNet
    stage-2 shape), no residual, no second source, activation none / ReLU."""
    return (spec.kind == "conv" and spec.R == 3 and spec.S == 3 and spec.stride == 1 and spec.pad == 1
            and spec.Cc == 128 and spec.cout == 128 and spec.K == 1152 and spec.K1 is None
            and residual is None and x2 is None and spec.act in (ACT_NONE, ACT_RELU)
            and x.dim() == 4 and x.shape[2] == 28 and x.shape[3] >= 128 and x.stride(3) == 1
            and x.stride(2) % 8 == 0 and (out is None or (out.stride(3) == 1 and out.stride(2) % 8 == 0)))


def patchw_weight(spec: ConvSpec) -> torch.Tensor:
    """[4, 9, 8, 64, 8] MFMA fragment image of a 3x3 128 -> 128 weight for conv_patchw.hip:
    (32-channel chunk, tap, 16-output-channel block, lane = 16 (k group) + output row, 8
    channels) — each (chunk, tap) block is the 8 KB the kernel streams per step.  Cached on the
    spec and re-derived in place when the weight changes (as patch_weight)."""
    key = (spec.weight.data_ptr(), spec.weight._version)
    cached = getattr(spec, "_patchw_w", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    w = spec.weight.view(8, 16, 9, 4, 4, 8)                  # [nb, fr, tap, chunk, fq, e]
    img = w.permute(3, 2, 0, 4, 1, 5).reshape(4, 9, 8, 64, 8)
    if cached is not None:
        cached[1].copy_(img)
        img = cached[1]
    else:
        img = img.contiguous()
    spec._patchw_w = (key, img)
    return img


def refresh_derived(spec: ConvSpec) -> None:
    """Re-derive, in place, every lazily built weight image this spec already holds (patch /
    patchw / rows kernels).  Called by ``models.weights.load_state_dict``: a captured hipGraph
    replays these images without re-entering Python, so they cannot wait for the next eager call."""
    for attr, derive in (("_patch_w", patch_weight), ("_patchw_w", patchw_weight), ("_rows_w", rows_weight)):
        if getattr(spec, attr, None) is not None:
            derive(spec)


def _rows_strided(t: torch.Tensor | None, B: int, H: int) -> bool:
    return (t is not None and t.dim() == 4 and t.shape[0] == B and t.shape[1] == H and t.shape[2] == 80
            and t.stride(3) == 1 and t.stride(2) % 8 == 0 and t.stride(1) == 80 * t.stride(2)
            and t.stride(0) == H * t.stride(1))


def rows_variant_ok(spec: ConvSpec, x: torch.Tensor, residual=None, x2=None, out=None) -> bool:
    """Whether the row-stream kernel (variant 17, conv_rows.hip) applies: a 3x3 / stride 1 / pad 1
    conv 32 -> 32 channels on 80-wide NHWC views with uniformly strided rows (YOLOv8-n's C2f
    bottleneck convs at the P3 level), activation none / ReLU / SiLU, optional residual."""
    if not (spec.kind == "conv" and spec.R == 3 and spec.S == 3 and spec.stride == 1 and spec.pad == 1
            and spec.Cc == 32 and spec.cout == 32 and spec.K1 is None and x2 is None
            and spec.act in (ACT_NONE, ACT_RELU, ACT_SILU) and x.dim() == 4):
        return False
    B, H = x.shape[0], x.shape[1]
    return (_rows_strided(x, B, H) and (residual is None or _rows_strided(residual, B, H))
            and (out is None or _rows_strided(out, B, H)))


def rows_weight(spec: ConvSpec) -> torch.Tensor:
    """[9, 2, 64, 8] MFMA fragment image of a 3x3 32 -> 32 weight for conv_rows.hip: (tap,
    16-output-channel block, lane = 16 (k group) + output row, 8 channels).  Cached on the spec
    (re-derived in place when the weight changes)."""
    key = (spec.weight.data_ptr(), spec.weight._version)
    cached = getattr(spec, "_rows_w", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    w = spec.weight[:, :288].reshape(2, 16, 9, 4, 8)      # [j, fr, tap, fq, e]
    img = w.permute(2, 0, 3, 1, 4).reshape(9, 2, 64, 8)
    if cached is not None:
        cached[1].copy_(img)
        img = cached[1]
    else:
        img = img.contiguous()
    spec._rows_w = (key, img)
    return img


def pw_variant_ok(spec: ConvSpec, x: torch.Tensor, x2: torch.Tensor | None = None):
    """Whether the persistent pointwise kernels (conv_pw.hip) apply to a 1x1 / stride 1
    single-source conv with 16-byte aligned pixel rows: ``True`` for variant 12 only (K % 256 == 0,
    Cout % 128 == 0), ``"resident"`` for variants 12 and 13 (K = 256 / 512), ``"resident_only"``
    for variant 13 alone (K = 128, Cout % 256 == 0: the 256 x 128 resident weight block), ``"dual"``
    for variant 13 as a fused stage-2 projection (128 main + 256 strided shortcut columns)."""
    if x2 is not None:
        return "dual" if (spec.kind != "stem" and spec.K1 == 128 and spec.K == 384 and spec.Cc == 128
                          and spec.R == 1 and spec.S == 1 and spec.stride == 1 and spec.pad == 0
                          and spec.cout % 128 == 0 and x.stride(2) % 8 == 0 and x2.stride(2) % 8 == 0) else False
    if not (spec.kind != "stem" and x2 is None and spec.K1 is None and spec.R == 1 and spec.S == 1
            and spec.stride == 1 and spec.pad == 0 and spec.Cc == spec.K and x.stride(2) % 8 == 0):
        return False
    if spec.K == 128:
        return "resident_only" if spec.cout % 256 == 0 else False
    if spec.K % 256 or spec.cout % 128:
        return False
    return "resident" if spec.K in (256, 512) else True


def narrow_variant_ok(spec: ConvSpec, x2: torch.Tensor | None = None) -> bool:
    """Whether the direct narrow-layer kernel (variant 7, conv_narrow.hip) applies: a 3x3 / pad 1
    / stride 1-2 or 1x1 / stride 1 conv with 16 or 32 input and output channels, no second source."""
    shape_ok = ((spec.R == 3 and spec.S == 3 and spec.pad == 1 and spec.stride in (1, 2))
                or (spec.R == 1 and spec.S == 1 and spec.pad == 0 and spec.stride == 1))
    return (spec.kind != "stem" and x2 is None and spec.K1 is None and shape_ok
            and spec.Cc in (16, 32) and spec.cout in (16, 32))


def _tune(key, M, cout, launch, buf_ok=False, narrow_ok=False, patch_ok=False, pw_ok=False, has_res=False,
          patchw_ok=False, rows_ok=False):
    if cout <= 32:
        cands = [t + (0,) for t in NARROW_TILES]
        if narrow_ok:
            cands.append((8, 32, 7))         # variant 7: 8 x 32 output pixels per workgroup
            cands.append((16, 32, 7))        #            16 x 32
            cands.append((8, 64, 7))         # bn = 64: Cc-32 weights held in registers, not LDS
            cands.append((16, 64, 7))
        if rows_ok:
            cands.append((1, 32, 17))        # variant 17: persistent row stream (80-wide 32 -> 32 3x3)
    else:
        cands = [t + (0,) for t in TILES] + [t + (1,) for t in TILES]
        if cout in GLDS_EXACT_N:
            cands += [t + (1,) for t in ((128, cout), (256, cout))]
        if buf_ok:
            cands += [t + (2,) for t in TILES + BUF_WIDE_TILES] + [t + (3,) for t in BUF_OCC_TILES]
            cands += [t + (4,) for t in PERSIST_TILES]
            if 5 in _EXTRA:
                # variant 5 wins some ResNet layers in isolation, but the two-lane bench is ~1 % faster
                # without it (90.3k vs 91.4k frames/s, 5 + 5 interleaved runs on two boxes,
                # scripts/r5_skip_ab.sh; YOLO / Whisper never pick it): opt-in, AIKO_CONV_EXTRA=5
                cands += [t + (5,) for t in MF32_TILES]
            cands += [t + (8,) for t in WIDE8_TILES] + [t + (9,) for t in WIDE_OCC_TILES]
            if 19 in _EXTRA:
                cands += [t + (19,) for t in WIDE4_OCC_TILES]
            # variant 20: at B=320 the ResNet bench ran 1 % faster without it (89.8k vs 90.7k,
            # round 5, scripts/r5_skip_ab.sh); at the round-6 default B=640, interleaved on two
            # boxes: 94.6k / 94.2k with vs 93.2k / 93.2k without, then 92.63-92.70k vs
            # 92.64-92.86k (YOLOv8-n 50.0k both): default again, AIKO_CONV_SKIP=20 leaves it out
            if cout <= 2048 and not has_res:
                cands += [t + (20,) for t in WIDE_PERS_TILES]
            elif cout <= 2048 and key[2] >= 192:   # with a residual: 3-slot forms
                cands += [t + (20,) for t in WIDE_PERS_TILES if t != (256, 256)]
            if cout in EXACT_N:
                cands += [(256, cout, 18), (128, cout, 18)]
            # variants 6 and 11 were never the tuner's pick on any layer measured (rounds 3-4):
            # out of default tuning (setup time), kept for other shapes behind AIKO_CONV_EXTRA=6,11
            if 6 in _EXTRA:
                cands += [t + (6,) for t in WIDE4_TILES]
            if 11 in _EXTRA:
                cands += [t + (11,) for t in WIDE_DEEP_TILES]

        if patch_ok:
            cands.append((8, 64, 10))        # variant 10: tile fixed by the kernel (8 rows x W)
        if patchw_ok:
            cands.append((392, 128, 16))     # variant 16: 14-row patch tiles, streamed weights
        if pw_ok and pw_ok not in ("resident_only", "dual"):
            cands.append((128, 128, 12))     # variant 12: persistent pointwise GEMM (conv_pw.hip)
        if pw_ok in ("resident", "resident_only") or (pw_ok == "dual" and not has_res and _PW_DUAL):
            cands.append((64, 128, 13))      # variant 13: the same with the weight block resident in LDS
            if has_res and _PW_AB:
                cands.append((64, 128, 14))  # variant 14: variant 13 with each tile's residual issued at its own tile
    skip = {int(v) for v in __import__("os").environ.get("AIKO_CONV_SKIP", "").split(",") if v.strip()}
    if skip:                                   # A/B runs: exclude variants from the tuner
        cands = [t for t in cands if (t[2] if len(t) > 2 else 0) not in skip] or cands
    skip_t = {tuple(int(v) for v in e.split("x")) for e in __import__("os").environ.get("AIKO_CONV_SKIP_TILES", "").split(",")
              if e.strip()}                    # exact tiles, e.g. AIKO_CONV_SKIP_TILES=256x192x8
    if skip_t:
        cands = [t for t in cands if tuple(t) not in skip_t] or cands
    # each candidate: 2 warm launches, then the median of 5 individually timed ones (a 3-launch
    # sum was noisy enough to rank a 56 us kernel behind an 80 us one on a fresh box)
    best, best_t = None, None
    for t in cands:
        launch(t)
        launch(t)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for e0, e1 in evs:
            e0.record()
            launch(t)
            e1.record()
        evs[-1][1].synchronize()
        ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs)[2]
        if _TUNE_VERBOSE:
            print(f"[tune] M={M} N={cout} {t}: {ms * 1e3:.1f} us", flush=True)
        if best_t is None or ms < best_t:
            best, best_t = t, ms
    _tile_cache[key] = best
    return best


def pick_tile(M: int, cout: int) -> tuple[int, int]:
    """Block tile (BM, BN) for the igemm kernel: fill 256 CUs x 2 blocks first, then reuse."""
    if cout <= 32:
        return (256, 32) if math.ceil(M / 256) >= 512 else (128, 32)
    bn = 128 if cout % 128 == 0 else 64
    bm = 128
    tiles = math.ceil(M / bm) * math.ceil(cout / bn)
    if tiles < 512:
        bm = 64
        tiles = math.ceil(M / bm) * math.ceil(cout / bn)
        if tiles < 512 and bn == 128:
            bn = 64
    return bm, bn


def conv2d(x: torch.Tensor, spec: ConvSpec, residual: torch.Tensor | None = None,
           out: torch.Tensor | None = None, tile: tuple[int, int] | None = None,
           image_hw: tuple[int, int] | None = None, x2: torch.Tensor | None = None,
           residual_after_act: bool = False) -> torch.Tensor:
    """NHWC bf16 conv with fused bias / residual / activation on the MFMA igemm kernel.

    ``x`` is ``[B, H, W, C]`` — possibly a channel-slice view of a wider buffer (the pixel
    pitch is ``x.stride(2)``).  For a stem spec ``x`` is the zero-bordered ``[B, Hp, Wp, 4]``
    buffer from :func:`aiko_services_amd.ops.preprocess_frames` and ``image_hw`` the original
    image size.  ``residual`` (optional) has the output's shape.  ``x2`` is the second source of
    a :func:`fuse_shortcut` spec.  ``out`` may be a channel slice of a concat buffer.
    Returns ``out`` ``[B, Ho, Wo, Cout]``.
    """
    B, H, W, C = x.shape
    pitch = x.stride(2)
    if x.stride(3) != 1 or x.stride(1) != W * pitch or x.stride(0) != H * W * pitch:
        raise ValueError("conv2d: x must be NHWC with unit channel stride (a channel slice is fine)")
    if spec.kind == "stem":
        if image_hw is None:
            raise ValueError("conv2d: stem conv needs image_hw")
        Ho, Wo = spec.out_hw(*image_hw)
    else:
        if C < spec.Cc and pitch < spec.Cc:
            raise ValueError(f"conv2d: input has {C} channels, spec expects {spec.Cc}")
        Ho, Wo = spec.out_hw(H, W)
    M = B * Ho * Wo
    if out is None:
        out = torch.empty(B, Ho, Wo, spec.cout, dtype=torch.bfloat16, device=x.device)
    if spec.K1 is not None:
        if x2 is None or not x2.is_contiguous():
            raise ValueError("conv2d: fused-shortcut spec needs a contiguous x2")
        src2 = [spec.K1, x2.shape[1], x2.shape[2], x2.shape[3], spec.stride2]
    else:
        x2 = None
        src2 = [spec.K, 1, 1, 8, 1]
    act = spec.act | (ACT_RESIDUAL_AFTER if (residual is not None and residual_after_act) else 0)
    head = [H, W, pitch, spec.Cc, spec.R, spec.S, spec.stride, spec.pad, Ho, Wo, M,
            act, out.stride(2) if out.dim() == 4 else out.stride(0),
            0 if residual is None else (residual.stride(2) if residual.dim() == 4 else residual.stride(0))]

    def launch(t):
        # t = (BM, BN) or (BM, BN, variant): variant 1 = LDS-DMA kernel (needs the zero page),
        # 2 = buffer-LDS-DMA kernel
        v = t[2] if len(t) > 2 else 0
        if v == 10:
            if not patch_variant_ok(spec, x, residual, x2, out):
                raise ValueError("conv2d: variant 10 needs a 3x3/s1/p1 64->64 conv on a contiguous W<=56 input")
            torch.ops.aiko.conv3x3_patch_out(x, patch_weight(spec), spec.bias, out, spec.act, 0)
            return
        if v == 17:
            if not rows_variant_ok(spec, x, residual, x2, out):
                raise ValueError("conv2d: variant 17 needs a 3x3/s1/p1 32->32 conv on 80-wide row-strided views")
            torch.ops.aiko.conv3x3_rows_out(x, rows_weight(spec), spec.bias, residual, out, act, 0)
            return
        if v == 16:
            if not patchw_variant_ok(spec, x, residual, x2, out):
                raise ValueError("conv2d: variant 16 needs a 3x3/s1/p1 128->128 conv on a [B, H, 28, >=128] input")
            torch.ops.aiko.conv3x3_patchw_out(x, patchw_weight(spec), spec.bias, out, spec.act, 0)
            return
        torch.ops.aiko.conv_igemm_out(x, x2, spec.weight, spec.bias, residual, out,
                                      head + [t[0], t[1]] + src2 + [v], zero_page(x.device) if v == 1 else None)

    if tile is None:
        key = (M, spec.cout, spec.K, spec.R, spec.S, spec.stride, pitch, spec.K1, residual is not None, spec.Cc)
        tile = _tile_cache.get(key)
        if tile is None:
            if _tuning:
                tile = _tune(key, M, spec.cout, launch, buf_variant_ok(spec, x, x2), narrow_variant_ok(spec, x2),
                             patch_variant_ok(spec, x, residual, x2, out) and not residual_after_act,
                             pw_variant_ok(spec, x, x2), residual is not None,
                             patchw_variant_ok(spec, x, residual, x2, out) and not residual_after_act,
                             rows_variant_ok(spec, x, residual, x2, out))
            else:
                tile = pick_tile(M, spec.cout)
    launch(tile)
    return out


STEM_POOL_VARIANT = 0     # 0: 8x7 pooled tiles (4 workgroups/CU); 1: 8x14 (2 workgroups/CU)
# uint8 stem: 2 = the strip kernel (weights in registers for a 7-column strip of pooled tiles,
# horizontal max in DPP lanes): 126.6 us vs 136.1 us for the tile kernel at B=256 on MI355X;
# 3 (default) = the strip kernel with half-channel waves (124 VGPRs, 40.6 KB LDS: 4 workgroups
# per CU instead of 2, room for the other frame lane): 126-128 us vs 143-150 us for variant 2 on
# the same box, ResNet-50 bench 85.2k / 83.9k vs 81.7k / 83.0k interleaved; 4 = four rows per
# MFMA group (3 workgroups per CU), not faster
STEM_POOL_U8_VARIANT = 3


def stem_pool_weight(spec: ConvSpec) -> torch.Tensor:
    """[7, 64, 32] LDS image of a packed 7x7 stem weight for the fused kernel: filter row r,
    channel o, 16-byte chunk ``pos`` holds K columns ``r*32 + 8*(pos ^ ((o >> 2) & 2))`` (the
    swizzle that makes the kernel's A-fragment reads bank-conflict free).  Cached on the spec;
    when the weight tensor changes (``load_state_dict`` copies in place, bumping ``_version``)
    the image is re-derived INTO THE SAME TENSOR, so a hipGraph captured earlier replays the
    new weights instead of a stale (or freed) image."""
    key = (spec.weight.data_ptr(), spec.weight._version)
    cached = getattr(spec, "_stem_pool_w", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    w = spec.weight.view(64, 8, 4, 8)[:, :7].permute(1, 0, 2, 3)         # [r, o, q, j]
    o = torch.arange(64, device=w.device)
    q = torch.arange(4, device=w.device)[None, :] ^ ((o[:, None] >> 2) & 2)  # [o, pos]
    img = torch.gather(w, 2, q[None, :, :, None].expand(7, 64, 4, 8)).reshape(7, 64, 32)
    if cached is not None:
        cached[1].copy_(img)
        img = cached[1]
    else:
        img = img.contiguous()
    spec._stem_pool_w = (key, img)
    return img


def stem_pool(x: torch.Tensor, spec: ConvSpec, image_hw: tuple[int, int],
              out: torch.Tensor | None = None, variant: int | None = None) -> torch.Tensor:
    """ResNet stem fused with its max-pool: ``maxpool3x3/s2/p1(relu(stem7x7/s2(x) + b))`` in ONE
    kernel (``csrc/kernels/stem_pool.hip``) — the [B, H/2, W/2, 64] stem activation never
    reaches HBM.  ``x`` is the zero-bordered preprocess buffer, ``spec`` a 7x7/s2 ReLU stem
    with 64 output channels (``make_stem_spec``).  Bit-identical to ``conv2d`` + ``maxpool2d``."""
    if spec.kind != "stem" or spec.stem_k != 7 or spec.stride != 2 or spec.cout != 64 \
            or spec.act != ACT_RELU or spec.bias is None:
        raise ValueError("stem_pool: needs a 7x7/s2 ReLU stem spec with 64 channels and a bias")
    Ho, Wo = spec.out_hw(*image_hw)
    Hm, Wm = (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1
    if out is None:
        out = torch.empty(x.shape[0], Hm, Wm, 64, dtype=torch.bfloat16, device=x.device)
    torch.ops.aiko.stem_pool_out(x, stem_pool_weight(spec), spec.bias, out, Ho, Wo,
                                 STEM_POOL_VARIANT if variant is None else variant)
    return out


def stem_pool_u8_weight(spec: ConvSpec, std) -> torch.Tensor:
    """The fused stem's weight image (:func:`stem_pool_weight`) with input channel c scaled by
    1 / (255 std_c): the uint8 variant feeds ``pixel - 255 mean_c`` instead of the normalised
    value.  Cached and re-derived in place like the unscaled image."""
    key = (spec.weight.data_ptr(), spec.weight._version, tuple(float(v) for v in std))
    cached = getattr(spec, "_stem_pool_u8_w", None)
    if cached is not None and cached[0] == key:
        return cached[1]
    base = stem_pool_weight(spec).float().view(7, 64, 4, 8)               # [r, o, chunk, 2 px x 4 ch]
    scale = torch.tensor([1.0 / (255.0 * float(v)) for v in std] + [0.0], device=base.device)
    img = (base.view(7, 64, 4, 2, 4) * scale).to(torch.bfloat16).view(7, 64, 32)
    if cached is not None:
        cached[1].copy_(img)
        img = cached[1]
    else:
        img = img.contiguous()
    spec._stem_pool_u8_w = (key, img)
    return img


def stem_pool_u8(frames: torch.Tensor, spec: ConvSpec, mean, std, out: torch.Tensor | None = None,
                 variant: int | None = None) -> torch.Tensor:
    """:func:`stem_pool` fed with uint8 frames ``[B, H, W, 3]`` (the stem's own image size,
    ``W % 4 == 0``): the kernel normalises while it fills its LDS patch — no pre-processing
    kernel and no bf16 stem buffer round trip through HBM.  ``mean`` / ``std`` as for
    :func:`ops.vision.preprocess_frames` (fractions of 255)."""
    if spec.kind != "stem" or spec.stem_k != 7 or spec.stride != 2 or spec.cout != 64 \
            or spec.act != ACT_RELU or spec.bias is None:
        raise ValueError("stem_pool_u8: needs a 7x7/s2 ReLU stem spec with 64 channels and a bias")
    B, H, W, _ = frames.shape
    Ho, Wo = spec.out_hw(H, W)
    Hm, Wm = (Ho - 1) // 2 + 1, (Wo - 1) // 2 + 1
    if out is None:
        out = torch.empty(B, Hm, Wm, 64, dtype=torch.bfloat16, device=frames.device)
    torch.ops.aiko.stem_pool_u8_out(frames, stem_pool_u8_weight(spec, std), spec.bias, out,
                                    [255.0 * float(m) for m in mean],
                                    STEM_POOL_U8_VARIANT if variant is None else variant)
    return out


LINEAR_SPLITK = 4     # K slices of the split-K linear (linear_splitk.hip)
_LINEAR_SPLITK_ON = __import__("os").environ.get("AIKO_FC_SPLITK", "1") != "0"


def linear_splitk_ok(x: torch.Tensor, spec: ConvSpec, residual=None) -> bool:
    """Whether the split-K kernel applies: no activation / residual, K a multiple of 32 S, a
    short M (the tile grid over M x N alone would not fill the chip) and N % 4 == 0."""
    return (residual is None and spec.act == ACT_NONE and spec.K % (32 * LINEAR_SPLITK) == 0
            and spec.cout % 4 == 0 and x.shape[0] <= 2048 and spec.K >= 1024 and x.stride(1) == 1
            and x.stride(0) % 8 == 0)


def linear(x: torch.Tensor, spec: ConvSpec, out: torch.Tensor | None = None,
           residual: torch.Tensor | None = None, work: torch.Tensor | None = None) -> torch.Tensor:
    """``[B, K] @ W^T + b`` on the same kernel (1x1 "image").  With ``work`` (fp32, >= S*B*N
    elements, private to the calling stream) a short-M / long-K layer runs split-K
    (linear_splitk.hip: S x more workgroups, deterministic two-kernel reduction)."""
    B, K = x.shape
    if out is None:
        out = torch.empty(B, spec.cout, dtype=torch.bfloat16, device=x.device)
    if (work is not None and _LINEAR_SPLITK_ON and linear_splitk_ok(x, spec, residual)
            and work.numel() >= LINEAR_SPLITK * B * spec.cout):
        torch.ops.aiko.linear_splitk_out(x, spec.weight.view(spec.cout, -1), spec.bias, work, out, spec.K,
                                         LINEAR_SPLITK)
        return out
    bm, bn = pick_tile(B, spec.cout)
    geom = [1, 1, x.stride(0), spec.Cc, 1, 1, 1, 0, 1, 1, B, spec.act, out.stride(0),
            0 if residual is None else residual.stride(0), bm, bn, spec.K, 1, 1, 8, 1]
    torch.ops.aiko.conv_igemm_out(x, None, spec.weight, spec.bias, residual, out, geom)
    return out




def conv_tail_ok(x: torch.Tensor, spec: ConvSpec, spec2: ConvSpec) -> bool:
    """Can ``spec`` (a 3x3 conv to N = 64, 80 or 128 channels, any stride) and the following 1x1
    ``spec2`` (N -> N, bias, no activation or SiLU) run as ONE ``conv_glds`` launch with the 1x1
    in its epilogue (the YOLOv8 detect head's box and class branches; l3 -> l4's and l5 -> l6's
    C2f cv1)?"""
    n = spec.cout
    return (spec.kind == "conv" and spec.R == spec.S == 3 and spec.K1 is None and n in (64, 80, 128)
            and spec.bias is not None and x.dim() == 4 and x.shape[3] == spec.Cc and spec.Cc % 8 == 0
            and x.stride(3) == 1 and x.stride(2) % 8 == 0
            and spec2.kind == "conv" and spec2.R == spec2.S == 1 and spec2.stride == 1 and spec2.pad == 0
            and spec2.K1 is None and spec2.Cc == n and spec2.cout == n and spec2.bias is not None
            and spec2.act in (ACT_NONE, ACT_SILU) and spec2.weight.shape[1] >= (n + 31) // 32 * 32)


def conv2d_tail(x: torch.Tensor, spec: ConvSpec, spec2: ConvSpec, out: torch.Tensor) -> torch.Tensor:
    """``out = conv1x1(act(conv(x, spec)), spec2)`` in one launch (``conv_glds.hip`` TAIL: the
    activated 3x3 tile stays in LDS and feeds the 1x1's MFMAs; it is never written to HBM).
    ``x`` / ``out`` may be channel-slice views.  See :func:`conv_tail_ok`."""
    if not conv_tail_ok(x, spec, spec2):
        raise ValueError("conv2d_tail: shapes not eligible (see conv_tail_ok)")
    torch.ops.aiko.conv_glds_tail_out(x, spec.weight, spec.bias, spec2.weight, spec2.bias, out, spec.R, spec.stride,
                                      spec.pad, spec.act, spec2.act, zero_page(x.device))
    return out


def chain_ok(spec3: ConvSpec, spec1: ConvSpec) -> bool:
    """Can ``spec3`` (1x1 expansion, identity residual) and the next block's ``spec1`` (1x1
    reduction) run as one ``conv_chain`` launch?"""
    def one_by_one(s):
        return s.kind == "conv" and s.R == 1 and s.S == 1 and s.stride == 1 and s.K1 is None and s.bias is not None
    # (K1, N1) -> allowed N2.  Stage 2 -> 128 runs on conv_chain2.hip (both weight matrices
    # resident in registers).  Measured and removed (round 6 pruning, numbers in profiles/):
    # stage 2 -> 256 on the register-staged kernel (spills: 519 vs 200 us unchained) and the
    # stage-3 chain (conv_chain3: 179 vs 101 us, profiles/chain3_stage3_r5.txt).
    shapes = {(64, 256): (64, 128), (128, 512): (128,)}
    k1, n1 = spec3.weight.shape[1], spec3.weight.shape[0]
    return (one_by_one(spec3) and one_by_one(spec1) and spec3.cin == k1 and (k1, n1) in shapes
            and spec1.cin == n1 and spec1.weight.shape[1] == n1 and spec1.cout in shapes[(k1, n1)]
            and spec3.act == ACT_RELU and spec1.act == ACT_RELU)


def chain_dual_ok(fused: ConvSpec, spec1: ConvSpec) -> bool:
    """A block's first conv3 with its fused 1x1 stride-1 projection shortcut (K = 64 + 64 -> 256)
    followed by the next block's 1x1 reduction to 64 channels."""
    return (fused.K1 == 64 and fused.stride2 == 1 and fused.weight.shape == (256, 128) and fused.R == 1
            and fused.S == 1 and fused.stride == 1 and fused.bias is not None and fused.act == ACT_RELU
            and spec1.kind == "conv" and spec1.R == 1 and spec1.S == 1 and spec1.stride == 1 and spec1.K1 is None
            and spec1.weight.shape == (64, 256) and spec1.bias is not None and spec1.act == ACT_RELU)


def bneck_ok(x: torch.Tensor, conv1: ConvSpec, conv2: ConvSpec, conv3: ConvSpec) -> bool:
    """Can this ResNet bottleneck run as ONE ``bneck_fused`` launch (``bneck_fused.hip``)?
    Stage-1 geometry: x NHWC [B, H, 56, 256] with an identity residual (``conv3`` 64 -> 256), or
    x [B, H, 56, 64] with ``conv3`` the K-concatenated conv3 + 1x1 projection (``fuse_shortcut``:
    weight [256, 128]); conv1 1x1 -> 64, conv2 3x3 / stride 1 / pad 1 64 -> 64; every conv with
    a bias and ReLU."""
    def relu_bias(s):
        return s.kind == "conv" and s.bias is not None and s.act == ACT_RELU
    if not (x.dim() == 4 and x.is_contiguous() and x.dtype == torch.bfloat16 and x.shape[2] == 56
            and relu_bias(conv1) and relu_bias(conv2) and relu_bias(conv3)):
        return False
    cin = x.shape[3]
    k3 = 128 if cin == 64 else 64
    return (cin in (64, 256) and conv1.R == conv1.S == 1 and conv1.stride == 1 and conv1.K1 is None
            and tuple(conv1.weight.shape) == (64, cin) and conv2.R == conv2.S == 3 and conv2.stride == 1
            and conv2.pad == 1 and tuple(conv2.weight.shape) == (64, 576) and conv3.R == conv3.S == 1
            and conv3.stride == 1 and tuple(conv3.weight.shape) == (256, k3)
            and (conv3.K1 is None if cin == 256 else (conv3.K1 == 64 and conv3.stride2 == 1)))


def bneck_fused(x: torch.Tensor, conv1: ConvSpec, conv2: ConvSpec, conv3: ConvSpec, out: torch.Tensor | None = None,
                grid: int = 0) -> torch.Tensor:
    """A whole stage-1 ResNet bottleneck in one kernel: ``relu(conv3(relu(conv2(relu(conv1(x)))))
    + x)`` (identity block) or ``relu([conv2 out | x] . W3^T + b)`` with ``conv3`` the fused
    conv3 + projection (entry block).  The 64-channel intermediates never leave LDS.  Persistent:
    ``grid`` workgroups (0 = one per CU) each stream a contiguous range of the B * H output rows
    across image boundaries."""
    if not bneck_ok(x, conv1, conv2, conv3):
        raise ValueError("bneck_fused: shapes not eligible (see bneck_ok)")
    if out is None:
        out = torch.empty(*x.shape[:3], 256, dtype=torch.bfloat16, device=x.device)
    torch.ops.aiko.bneck_fused_out(x, conv1.weight, conv1.bias, conv2.weight, conv2.bias, conv3.weight,
                                   conv3.bias, out, grid)
    return out


def conv_chain(x: torch.Tensor, spec3: ConvSpec, residual: torch.Tensor | None, out_y: torch.Tensor,
               spec1: ConvSpec, out_z: torch.Tensor, grid: int = 0, x2: torch.Tensor | None = None):
    """``out_y = relu(conv1x1(x, spec3) + residual)``, ``out_z = relu(conv1x1(out_y, spec1))`` in
    one kernel (``conv_chain.hip``): the 256-channel ``out_y`` is written once and never read
    back.  All NHWC, contiguous.  With ``x2`` (and no residual) ``spec3`` is a fused-shortcut
    spec (:func:`chain_dual_ok`): ``out_y = relu([x | x2] . W^T + b)``."""
    ok = chain_dual_ok(spec3, spec1) if x2 is not None else chain_ok(spec3, spec1)
    if not ok:
        raise ValueError("conv_chain: shapes not eligible (chain_ok / chain_dual_ok)")
    torch.ops.aiko.conv_chain_out(x, spec3.weight, spec3.bias, residual, out_y, spec1.weight, spec1.bias,
                                  out_z, grid, x2)
    return out_y, out_z
