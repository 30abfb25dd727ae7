"""Transformer ops on the CDNA4 kernels: fp8 (OCP e4m3fn) linear layers on the block-scaled
MFMA, fused LayerNorm + per-token fp8 quantisation, flash attention forward
(``csrc/kernels/gemm_fp8.hip``, ``csrc/kernels/attention.hip``).

Quantisation scheme (inference):
* weights: per output channel, ``s_w[n] = amax(|W[n, :]|) / 448``, stored e4m3fn [N, K]
  (K zero-padded to a multiple of 128), quantised once at load;
* activations: per row (token), ``s_x[m] = amax(|x[m, :]|) / 448``, produced by the kernel that
  writes the activation (LayerNorm, or the quantise pass over attention / MLP outputs);
* the GEMM multiplies e4m3 x e4m3 on ``v_mfma_scale_f32_16x16x128_f8f6f4`` and applies
  ``s_x[m] * s_w[n]`` (+ bias, GELU, residual) in its fp32 epilogue.
"""
from __future__ import annotations

import os

from dataclasses import dataclass, field

import torch

from . import conv as _conv

__all__ = ["Fp8Linear", "make_fp8_linear",
           "quantize_rows_ref", "linear_fp8", "rownorm",
           "attention", "ACT_NONE", "ACT_RELU", "ACT_SILU", "ACT_GELU", "FP8_MAX", "pick_tile"]

ACT_NONE, ACT_RELU, ACT_SILU, ACT_GELU = 0, 1, 2, 3
FP8_MAX = 448.0
FP8 = torch.float8_e4m3fn


def _round_up(v, m):
    return (v + m - 1) // m * m


@dataclass
class Fp8Linear:
    weight: torch.Tensor            # uint8 view of e4m3fn [N, Kp]
    scale: torch.Tensor             # fp32 [N]
    bias: torch.Tensor | None       # fp32 [N]
    n: int
    k: int
    ref_weight: torch.Tensor | None = field(default=None, repr=False)   # dequantised fp32 [N, K]
    cs: torch.Tensor | None = field(default=None, repr=False)   # LayerNorm-folded: sum_k W[n, k] fp32 [N]

    def to(self, device):
        self.weight = self.weight.to(device)
        self.scale = self.scale.to(device)
        if self.bias is not None:
            self.bias = self.bias.to(device)
        if self.cs is not None:
            self.cs = self.cs.to(device)
        return self

    @property
    def K(self):
        return self.weight.shape[1]


def make_fp8_linear(w: torch.Tensor, bias: torch.Tensor | None = None, device=None) -> Fp8Linear:
    """Quantise an fp32 [N, K] weight per output channel to e4m3fn."""
    n, k = w.shape
    w = w.float()
    amax = w.abs().amax(dim=1).clamp(min=1e-12)
    scale = amax / FP8_MAX
    q = (w / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    kp = _round_up(k, 128)
    qp = torch.zeros(n, kp, dtype=torch.uint8)
    qp[:, :k] = q.view(torch.uint8)
    ref = q.float() * scale[:, None]
    lin = Fp8Linear(qp.contiguous(), scale.contiguous(), None if bias is None else bias.float().contiguous(),
                    n, k, ref)
    return lin.to(device) if device is not None else lin


def dequant_fp8_linear(lin: Fp8Linear) -> torch.Tensor:
    """fp32 [N, K] values of ``lin``'s quantised weight (its ``ref_weight`` when held)."""
    if lin.ref_weight is not None:
        return lin.ref_weight.float()
    return lin.weight[:, :lin.k].view(FP8).float() * lin.scale.float()[:, None]


def quantize_rows_ref(x: torch.Tensor):
    """Reference per-row e4m3 quantisation: (q as uint8, scale fp32 [M])."""
    x = x.float()
    amax = x.abs().amax(dim=1)
    s = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    q = (x / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q.view(torch.uint8), s


def pick_tile(M: int, N: int) -> tuple[int, int]:
    bn = 128 if N % 128 == 0 else 64
    bm = 128
    if -(-M // bm) * -(-N // bn) < 512:
        bm = 64
    return bm, bn


def mx_buffers(M: int, K: int, device) -> tuple[torch.Tensor, torch.Tensor]:
    """Storage for an MX-fp8 activation: e4m3 bytes [M, K] and E8M0 scales, one per 32
    consecutive K values, laid out [K/128, rows, 4] (rows = M rounded up to 128)."""
    rows = -(-M // 128) * 128
    return (torch.empty(M, K, dtype=torch.uint8, device=device),
            torch.full((K // 128, rows, 4), 127, dtype=torch.uint8, device=device))


def mx_dequant(q: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """fp32 values of an MX-fp8 activation (test reference)."""
    M, K = q.shape
    v = q.view(torch.float8_e4m3fn).float().view(M, K // 128, 4, 32)          # [m, chunk, block, j]
    e = sc[:, :M].permute(1, 0, 2).float() - 127.0                             # [m, chunk, block]
    return (v * torch.exp2(e)[..., None]).reshape(M, K)


def mx_quantize_ref(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Reference MX-fp8 quantisation of fp32 [M, K] (same block layout and E8M0 rule)."""
    M, K = x.shape
    v = x.float().reshape(M, K // 128, 4, 32)
    amax = v.abs().amax(dim=3)                                                 # [m, chunk, block]
    t = (amax / FP8_MAX).clamp(min=2.0 ** -126)
    e = torch.ceil(torch.log2(t)).clamp(-126, 127)
    e = torch.where(amax == 0, torch.full_like(e, -126.0), e)
    q = (v / torch.exp2(e)[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    rows = -(-M // 128) * 128
    sc = torch.full((K // 128, rows, 4), 127, dtype=torch.uint8)
    sc[:, :M] = (e + 127).to(torch.uint8).permute(1, 0, 2)
    return q.reshape(M, K).view(torch.uint8), sc


def linear_fp8(xq: torch.Tensor, xs: torch.Tensor | None, lin: Fp8Linear, out: torch.Tensor | None = None,
               residual: torch.Tensor | None = None, act: int = ACT_NONE, tile=None,
               x_mx: torch.Tensor | None = None, out_mx: tuple | None = None) -> torch.Tensor | None:
    """``act(xs[m] * s_w[n] * (xq @ Wq^T) + bias) + residual`` -> bf16 [M, N].
    ``xq`` uint8 [M, K] (row pitch may exceed K), ``xs`` fp32 [M] per-row scales, or ``x_mx``
    (E8M0 block scales from :func:`mx_buffers`) for an MX-fp8 activation.  ``out_mx`` = (q, sc)
    quantises the output to MX-fp8 in the epilogue instead of writing bf16 (no residual)."""
    M = xq.shape[0]
    if xq.shape[1] != lin.K:
        raise ValueError(f"linear_fp8: activation K {xq.shape[1]} != weight K {lin.K}")
    if out is None and out_mx is None:
        out = torch.empty(M, lin.n, dtype=torch.bfloat16, device=xq.device)
    mx = x_mx is not None or out_mx is not None
    if tile is None:
        key = (M, lin.n, lin.K, xq.stride(0), residual is not None, act, x_mx is not None, out_mx is not None)
        tile = _tile_cache.get(key)
        if tile is None:
            launch = lambda t: _launch(xq, xs, lin, out, residual, act, t, x_mx, out_mx)  # noqa: E731
            if _conv._tuning:
                tile = _tune_fp8(key, launch, mx)
            else:
                tile = (128, 128, 1) if mx else pick_tile(M, lin.n) + (1,)
    _launch(xq, xs, lin, out, residual, act, tile, x_mx, out_mx)
    return out


def _launch(xq, xs, lin, out, residual, act, t, x_mx=None, out_mx=None):
    v = t[2] if len(t) > 2 else 0
    yq, ysc = out_mx if out_mx is not None else (None, None)
    torch.ops.aiko.gemm_fp8_out(xq, None if x_mx is not None else xs, lin.weight, lin.scale, lin.bias, residual,
                                out, act, t[0], t[1], v, _conv.zero_page(xq.device) if v else None,
                                x_mx, yq, ysc)


_tile_cache: dict = {}
FP8_TILES = ((128, 128), (128, 64), (64, 128), (64, 64))


def _tune_fp8(key, launch, mx=False):
    """Pick (BM, BN, variant) by measurement, like ``ops.conv.autotune`` (shares its switch)."""
    best, best_t = None, None
    if mx:                               # MX-fp8 in/out: LDS-DMA kernels, whole 128-wide K chunks
        cands = [(128, 128, 1), (64, 128, 1)]
    else:
        cands = [tt + (v,) for tt in FP8_TILES for v in (0, 1)]
        if key[1] % 128 == 0:
            cands.append((256, 128, 2))  # 8-wave LDS-DMA kernel (one workgroup per CU)
    if key[1] % 256 == 0:
        cands.append((256, 256, 3))      # 256 x 256 tile, 8 waves of 128 x 64 (MX in / out too)
        if key[1] <= 3072 and (
                (not key[4] and not key[6]) or (key[4] and key[6] and key[5] == 0 and not key[7])):
            # persistent 256 x 256, register-direct epilogue (no residual / MX input, or MX input +
            # residual with no activation: the out-projection / fc2 form).  Measured at
            # the 14-stream shapes (M = 21014, K = 768): qkv 62.8 -> 56.8 us (1.31 PF), fc1 + GELU +
            # MX out 104.8 -> 97.7 us against the best earlier kernel
            cands.append((256, 256, 4))
        if key[1] <= 3072 and (
                (not key[4] and not key[6] and key[5] in (0, 3) and (key[5] == 3 or not key[7]))
                or (key[4] and key[6] and key[5] == 0 and not key[7])):
            # persistent 128 x 256 (two row tiles per CU at N = 768): no residual / MX input, or the
            # out-projection / fc2 form (MX-fp8 A + residual, no activation, bf16 out).  Isolated
            # at the 14-stream shapes: out-proj 27.8 vs 28.6 us (best earlier), fc2 68.9 vs 62.0,
            # qkv 57.3 vs 51.6 (variant 4) — the tuner keeps it where it wins (scripts/fp8_v5_check.sh)
            cands.append((128, 256, 5))
    # AIKO_FP8_SKIP="256x256x4,128x256x5": candidates (BM x BN x variant) the tuner leaves out
    skip = {s.strip() for s in os.environ.get("AIKO_FP8_SKIP", "").split(",") if s.strip()}
    cands = [t for t in cands if "x".join(map(str, t)) not in skip] or cands
    for t in cands:
        try:
            launch(t)
            launch(t)
        except RuntimeError:
            continue
        times = []
        for _ in range(5):               # median of individually timed launches
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch(t)
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1))
        ms = sorted(times)[2]
        if _conv._TUNE_VERBOSE:
            print(f"[tune fp8] M={key[0]} N={key[1]} K={key[2]} {t}: {ms * 1e3:.1f} us", flush=True)
        if best_t is None or ms < best_t:
            best, best_t = t, ms
    _tile_cache[key] = best
    return best


def rownorm(x: torch.Tensor, gamma=None, beta=None, eps: float = 1e-5, out: torch.Tensor | None = None,
            q: torch.Tensor | None = None, qs: torch.Tensor | None = None):
    """LayerNorm (when ``gamma``/``beta`` are given) of bf16 rows, writing bf16 ``out`` and/or
    per-row e4m3 ``q`` + scales ``qs`` in one pass."""
    torch.ops.aiko.rownorm_quant_out(x, gamma, beta, float(eps), out, q, qs)
    return out, q, qs


ATTN_WORKSPACE_BYTES = 40 << 20     # split-KV tail partials: <= 8 x 64 pieces x 256 rows x 66 fp32


def attention_workspace(device) -> torch.Tensor:
    """Zero-initialised scratch for :func:`attention`'s split-KV tail (fp32 partial outputs and
    per-item arrival counters, which the kernel re-arms): one per concurrently running stream."""
    return torch.zeros(ATTN_WORKSPACE_BYTES // 4, dtype=torch.float32, device=device)


def attention(q, k, v, out, batch: int, heads: int, T: int, Tpad: int, scale: float,
              work: torch.Tensor | None = None, out_mx: tuple | None = None):
    """Non-causal multi-head attention (head dim 64) over sequences of ``T`` tokens stored
    every ``Tpad`` rows; q/k/v may be column slices of one fused QKV buffer.  ``work``
    (:func:`attention_workspace`, private to the calling stream) lets the kernel cut the items
    of a partial last round into key ranges merged in-kernel.  ``out_mx`` = (q, sc) from
    :func:`mx_buffers`: the output is written as MX-fp8 (each head's 64 columns are two E8M0
    blocks, quantised in the epilogue) for an out-projection with ``x_mx`` — ``out`` is then
    not written."""
    oq, osc = out_mx if out_mx is not None else (None, None)
    torch.ops.aiko.attn_fwd_out(q, k, v, out, batch, heads, T, Tpad, float(scale), work, oq, osc)
    return out
