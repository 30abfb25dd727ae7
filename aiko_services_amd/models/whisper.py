"""Whisper audio encoder (tiny … large) on aiko_services_amd's CDNA4 kernels, fp8 weights.

The reference runs WhisperX / faster-whisper inside ``PE_WhisperX``
(``examples/speech/speech_elements.py:203-262``); BASELINE config 5 is the
Whisper-small encoder on streamed audio chunks with fp8 weights.  Execution per batch of clips
(one HIP stream, fixed buffers, hipGraph-capturable):

  audio fp32 [B, N] --logmel kernel--> bf16 [B*(F+2), 80] (zero frame border per clip)
  conv1 k3 (igemm, GELU) over the concatenated clips, written one row down so every clip's
        output lands inside its own zero border; border rows re-zeroed
  conv2 k3/s2 (igemm, GELU, + positional embedding as a post-activation residual): clip b's
        tokens are rows b*(T+1) .. b*(T+1)+T-1 — one spare row per clip, never attended to
  L x { LN1 + e4m3 quantise -> QKV fp8 GEMM (+bias) -> flash attention (bf16) ->
        e4m3 quantise -> out-proj fp8 GEMM (+bias, + residual in place) ->
        LN2 + quantise -> FC1 fp8 GEMM (+bias, GELU) -> quantise -> FC2 fp8 GEMM (+residual) }
  ln_post -> bf16 [B, T, d_model]

A LayerNorm folded across the GEMM pairs (row statistics from the producer's epilogue, the affine
folded into the consumer's weights) was built and measured in round 5: numerically equivalent but
slower (profiles/whisper_lnfold_r5.md), and removed in round 6.

Linear weights are e4m3fn with per-channel scales (see ``ops/transformer.py``); the convs and
attention run in bf16.  Random init (no checkpoints offline), deterministic per seed.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import torch

from ..ops import audio as AU
from ..ops import conv as C
from .weights import WeightsMixin
from ..ops import transformer as TR

# name: (d_model, layers, heads)
SIZES = {"tiny": (384, 4, 6), "base": (512, 6, 8), "small": (768, 12, 12),
         "medium": (1024, 24, 16), "large": (1280, 32, 20)}
N_MELS = 80
N_CTX = 1500                      # tokens for a 30 s window (3000 mel frames, conv stride 2)


def sinusoids(length: int, channels: int, max_timescale: float = 10000.0) -> torch.Tensor:
    inc = math.log(max_timescale) / (channels // 2 - 1)
    inv = torch.exp(-inc * torch.arange(channels // 2, dtype=torch.float32))
    t = torch.arange(length, dtype=torch.float32)[:, None] * inv[None, :]
    return torch.cat([torch.sin(t), torch.cos(t)], dim=1)


@dataclass
class Block:
    ln1: tuple
    qkv: TR.Fp8Linear
    out: TR.Fp8Linear
    ln2: tuple
    fc1: TR.Fp8Linear
    fc2: TR.Fp8Linear


class WhisperEncoder(WeightsMixin):
    """``encode(audio [B, N] fp32 16 kHz) -> bf16 [B, T, d_model]``, T = N / 320 (1500 for 30 s)."""

    def __init__(self, size: str = "small", seed: int = 0, device="cuda", n_ctx: int = N_CTX):
        self.device = torch.device(device)
        self.size = size
        d, L, H = SIZES[size]
        self.d, self.layers_n, self.heads = d, L, H
        self.n_ctx = n_ctx
        # attention writes MX-fp8 for the out-projection (no per-row quantisation pass)
        self.mx_attention = os.environ.get("AIKO_WHISPER_MX_ATTN", "1") != "0" and d % 128 == 0
        g = torch.Generator().manual_seed(seed)
        dev = self.device

        def rnd(*shape, fan_in):
            return torch.randn(*shape, generator=g) / math.sqrt(fan_in)

        def small(n):
            return 0.02 * torch.randn(n, generator=g)

        self.filters = AU.mel_filters(N_MELS).to(dev)
        self.conv1 = C.make_conv_spec(rnd(d, N_MELS, 3, 1, fan_in=3 * N_MELS), small(d), pad=0,
                                      act="gelu", device=dev)
        self.conv2 = C.make_conv_spec(rnd(d, d, 3, 1, fan_in=3 * d), small(d), stride=2, pad=0,
                                      act="gelu", device=dev)
        self.pos = sinusoids(n_ctx, d).to(dev, torch.bfloat16)
        self.blocks = []
        for _ in range(L):
            ln1 = (1.0 + 0.1 * torch.randn(d, generator=g), small(d))
            ln2 = (1.0 + 0.1 * torch.randn(d, generator=g), small(d))
            wqkv = rnd(3 * d, d, fan_in=d)
            bqkv = torch.cat([small(d), torch.zeros(d), small(d)])      # key projection has no bias
            blk = Block(tuple(t.to(dev) for t in ln1), TR.make_fp8_linear(wqkv, bqkv, dev),
                        TR.make_fp8_linear(rnd(d, d, fan_in=d), small(d), dev),
                        tuple(t.to(dev) for t in ln2),
                        TR.make_fp8_linear(rnd(4 * d, d, fan_in=d), small(4 * d), dev),
                        TR.make_fp8_linear(rnd(d, 4 * d, fan_in=4 * d), small(d), dev))
            self.blocks.append(blk)
        self.ln_post = ((1.0 + 0.1 * torch.randn(d, generator=g)).to(dev), small(d).to(dev))
        self._ws: dict = {}
        self.ws_tag = ""             # workspace key prefix (one workspace per frame lane)
        self._pos_ready: set = set()

    # ---- weights ---------------------------------------------------------------------------------
    def named_layers(self):
        yield "conv1", self.conv1
        yield "conv2", self.conv2
        for i, b in enumerate(self.blocks):
            yield f"blocks.{i}.ln1", b.ln1
            yield f"blocks.{i}.qkv", b.qkv
            yield f"blocks.{i}.out", b.out
            yield f"blocks.{i}.ln2", b.ln2
            yield f"blocks.{i}.fc1", b.fc1
            yield f"blocks.{i}.fc2", b.fc2
        yield "ln_post", self.ln_post

    def config(self) -> dict:
        return {"size": self.size, "n_ctx": self.n_ctx}

    # ---- workspace ------------------------------------------------------------------------------
    def _buf(self, key, shape, dtype=torch.bfloat16, zero=False):
        k = (self.ws_tag + key, tuple(shape), dtype)
        t = self._ws.get(k)
        if t is None:
            t = (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=self.device)
            self._ws[k] = t
        return t

    def release_workspace(self):
        self._ws.clear()
        self._pos_ready.clear()

    def tokens_for(self, n_samples: int) -> int:
        frames = n_samples // AU.HOP
        return (frames - 1) // 2 + 1

    def flops_per_clip(self, n_samples: int = 480000) -> int:
        T = self.tokens_for(n_samples)
        F = n_samples // AU.HOP
        d = self.d
        conv = 2 * F * 3 * N_MELS * d + 2 * T * 3 * d * d
        per_layer = 2 * T * d * (3 * d + d + 8 * d) + 4 * T * T * d
        return conv + self.layers_n * per_layer

    # ---- forward --------------------------------------------------------------------------------
    def encode(self, audio: torch.Tensor) -> torch.Tensor:
        B, N = audio.shape
        d, H = self.d, self.heads
        F = N // AU.HOP
        T = (F - 1) // 2 + 1
        if T > self.n_ctx:
            raise ValueError(f"{N} samples give {T} tokens > n_ctx {self.n_ctx}")
        if F % 2:
            raise ValueError("frame count must be even (clip length a multiple of 320 samples)")
        rows1 = F + 2                          # per-clip mel rows incl. zero border
        Tp = T + 1                             # per-clip token rows incl. one spare
        mel = self._buf("mel", (B * rows1, N_MELS), zero=True)
        AU.log_mel(audio, self.filters, mel, rows1, 1,
                   work=self._buf("mel_work", (B * F * N_MELS,), torch.float32),
                   gmax=self._buf("mel_max", (B,), torch.int32), frames=F)
        # conv1 over the concatenated clips; output shifted one row into a zero-bordered buffer
        h1 = self._buf("h1", (B * rows1, d))
        M1 = B * rows1 - 2
        C.conv2d(mel.view(1, B * rows1, 1, N_MELS), self.conv1, out=h1[1:1 + M1].view(1, M1, 1, d))
        if h1.is_cuda:
            torch.ops.aiko.zero_border_rows_(h1, rows1)     # per-clip zero border rows (one kernel)
        else:
            h1v = h1.view(B, rows1, d)
            h1v[:, 0].zero_()
            h1v[:, rows1 - 1].zero_()
        # conv2 (stride 2) + positional embedding -> residual stream x [B*Tp, d]
        x = self._buf("x", (B * Tp, d), zero=True)
        M2 = B * Tp - 1
        pos = self._buf(f"pos{T}", (B * Tp, d), zero=True)
        if (self.ws_tag, B, T) not in self._pos_ready:
            pos.view(B, Tp, d)[:, :T] = self.pos[:T]
            self._pos_ready.add((self.ws_tag, B, T))
        C.conv2d(h1.view(1, B * rows1, 1, d), self.conv2, out=x[:M2].view(1, M2, 1, d),
                 residual=pos[:M2].view(1, M2, 1, d), residual_after_act=True)
        M = B * Tp
        q8 = self._buf("q8", (M, d), torch.uint8)
        s8 = self._buf("s8", (M,), torch.float32)
        qkv = self._buf("qkv", (M, 3 * d))
        att = self._buf("att", (M, d), zero=True)
        aws = self._buf("attn_ws", (TR.ATTN_WORKSPACE_BYTES // 4,), torch.float32, zero=True)
        # fc1 -> fc2 hand-off in MX-fp8: the fc1 epilogue applies GELU and writes e4m3 + E8M0
        # block scales, fc2 feeds those scales straight to the scaled MFMA (no bf16 round trip,
        # no separate row-quantisation pass)
        u8, usc = self._ws.get((self.ws_tag + "u_mx", M, 4 * d)) or (None, None)
        if u8 is None:
            u8, usc = TR.mx_buffers(M, 4 * d, self.device)
            self._ws[(self.ws_tag + "u_mx", M, 4 * d)] = (u8, usc)
        # attention -> out-projection hand-off in MX-fp8 too: the attention epilogue quantises
        # each head's 64 columns (two E8M0 blocks) itself, so no per-row quantisation pass
        a8, asc = self._ws.get((self.ws_tag + "a_mx", M, d)) or (None, None)
        if a8 is None and self.mx_attention:
            a8, asc = TR.mx_buffers(M, d, self.device)
            self._ws[(self.ws_tag + "a_mx", M, d)] = (a8, asc)
        for blk in self.blocks:
            TR.rownorm(x, *blk.ln1, q=q8, qs=s8)
            TR.linear_fp8(q8, s8, blk.qkv, out=qkv)
            if self.mx_attention:
                TR.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], att, B, H, T, Tp, (d // H) ** -0.5,
                             work=aws, out_mx=(a8, asc))
                TR.linear_fp8(a8, None, blk.out, out=x, residual=x, x_mx=asc)
            else:
                TR.attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], att, B, H, T, Tp, (d // H) ** -0.5,
                             work=aws)
                TR.rownorm(att, q=q8, qs=s8)
                TR.linear_fp8(q8, s8, blk.out, out=x, residual=x)
            TR.rownorm(x, *blk.ln2, q=q8, qs=s8)
            TR.linear_fp8(q8, s8, blk.fc1, act=TR.ACT_GELU, out_mx=(u8, usc))
            TR.linear_fp8(u8, None, blk.fc2, out=x, residual=x, x_mx=usc)
        y = self._buf("y", (M, d))
        TR.rownorm(x, *self.ln_post, out=y)
        return y.view(B, Tp, d)[:, :T]

    __call__ = encode

    # ---- fp32 torch reference (tests only): same weights (fp8-dequantised), no activation quant --
    def reference_encode(self, audio: torch.Tensor) -> torch.Tensor:
        import torch.nn.functional as F
        from ..ops import reference as R
        mel = AU.log_mel_ref(audio.float(), self.filters, frames=audio.shape[1] // AU.HOP)  # [B, 80, F]
        x = mel.to(torch.bfloat16).float()
        w1 = self.conv1.ref_weight.to(x.device)[..., 0]          # [d, 80, 3]
        x = F.gelu(F.conv1d(x, w1, self.conv1.ref_bias.to(x.device), padding=1))
        w2 = self.conv2.ref_weight.to(x.device)[..., 0]
        x = F.gelu(F.conv1d(x, w2, self.conv2.ref_bias.to(x.device), stride=2, padding=1))
        x = x.transpose(1, 2)
        T = x.shape[1]
        x = x + self.pos[:T].float()
        d, H = self.d, self.heads
        for blk in self.blocks:
            h = F.layer_norm(x, (d,), blk.ln1[0], blk.ln1[1], 1e-5)
            qkv = h @ blk.qkv.ref_weight.T.to(h.device) + blk.qkv.bias
            q, k, v = qkv.split(d, dim=-1)
            B = x.shape[0]
            sh = lambda t: t.view(B, T, H, d // H).transpose(1, 2)  # noqa: E731
            a = F.scaled_dot_product_attention(sh(q), sh(k), sh(v))
            a = a.transpose(1, 2).reshape(B, T, d)
            x = x + a @ blk.out.ref_weight.T.to(a.device) + blk.out.bias
            h = F.layer_norm(x, (d,), blk.ln2[0], blk.ln2[1], 1e-5)
            h = F.gelu(h @ blk.fc1.ref_weight.T.to(h.device) + blk.fc1.bias)
            x = x + h @ blk.fc2.ref_weight.T.to(h.device) + blk.fc2.bias
        del R
        return F.layer_norm(x, (d,), self.ln_post[0], self.ln_post[1], 1e-5)
