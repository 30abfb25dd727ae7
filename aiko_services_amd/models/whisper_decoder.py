"""Whisper text decoder (tiny … large): greedy autoregressive transcription on the CDNA4 kernels.

The speech-to-text half of the reference's ``PE_WhisperX`` (``examples/speech/
speech_elements.py:203-262``: ``transcribe(audio, language="en")`` -> ``{"text": ...}``); the
encoder half is ``models/whisper.py``.  A batch of ``B`` audio windows decodes together, one
token per sequence per step, entirely on the device:

  prepare(features [B, T, d]):   per layer, cross-attention K|V = fp8 GEMM over the encoder
                                 rows (once per window)  -> kv_cross[l] bf16 [B*S, 2d]
  step():                        embed(ids, pos) -> x [B, d]
                                 L x { [LN + e4m3 + QKV GEMM] -> decode attention (appends K/V
                                       at pos into kv_self[l], attends 0..pos) -> [e4m3 + out
                                       GEMM + res] -> [LN + e4m3 + cross-Q GEMM] -> decode
                                       attention over kv_cross[l] -> [e4m3 + cross-out GEMM +
                                       res] -> [LN + e4m3 + fc1 GEMM + GELU] -> [e4m3 + fc2
                                       GEMM + res] }   ([...] = one dec_linear launch)
                                 [LN + e4m3 + logits GEMM (tied embedding)] -> argmax step
                                 (forced prompt, sticky end-of-text, pos += 1 on the device)

Every launch reads the step position from device memory, so ``step`` is captured once into a
hipGraph and replayed per token; the host only checks for "all sequences finished" every few
steps.  Linear weights are e4m3fn with per-channel scales (``ops/transformer.py``), attention
and the embeddings are bf16.  Random init (no checkpoints offline), deterministic per seed.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from ..ops import transformer as TR
from .weights import WeightsMixin
from .whisper import SIZES

N_VOCAB = 51865          # multilingual vocabulary
N_TEXT_CTX = 448
# special tokens of the multilingual tokenizer
EOT = 50257
SOT = 50258
LANG_EN = 50259
TRANSCRIBE = 50359
NO_TIMESTAMPS = 50363
SOT_SEQUENCE = (SOT, LANG_EN, TRANSCRIBE, NO_TIMESTAMPS)
_KC = 256                # keys per split of the decode-attention kernel (decode_ops.hip)


def attn_decode_work(B: int, H: int, maxlen: int) -> int:
    """fp32 elements of the decode-attention workspace (per-split partials; an upper bound of
    the kernel's own split choice)."""
    return B * H * (-(-maxlen // _KC)) * (64 + 2)


def dec_linear(x, lin: TR.Fp8Linear, out, ln: tuple | None = None, residual=None, act: int = TR.ACT_NONE,
               eps: float = 1e-5):
    """Decoder linear for a few rows: LayerNorm (``ln`` = (gamma, beta)) and per-row e4m3
    quantisation fused into the fp8 MFMA GEMM (``dec_linear_kernel``)."""
    g, b = ln if ln is not None else (None, None)
    torch.ops.aiko.dec_linear_out(x, g, b, float(eps), lin.weight, lin.scale, lin.bias, residual, out, act)
    return out


def attn_decode(q, k, v, out, B: int, H: int, S: int, T: int, scale: float, work,
                pos=None, knew=None, vnew=None):
    """Flash-decoding attention of one query row per sequence (head dim 64); see
    ``csrc/kernels/decode_ops.hip``.  With ``pos`` the new key/value rows are appended at
    row ``pos`` of every sequence's cache first and keys 0..pos are attended."""
    torch.ops.aiko.attn_decode_out(q, k, v, out, B, H, S, T, pos, knew, vnew, float(scale), work)
    return out


@dataclass
class DecoderBlock:
    ln1: tuple
    qkv: TR.Fp8Linear
    out: TR.Fp8Linear
    lnx: tuple
    cq: TR.Fp8Linear
    ckv: TR.Fp8Linear
    cout: TR.Fp8Linear
    ln2: tuple
    fc1: TR.Fp8Linear
    fc2: TR.Fp8Linear


class WhisperDecoder(WeightsMixin):
    """``transcribe(features [B, T, d]) -> int32 [B, n]`` greedy token ids (prompt included)."""

    def __init__(self, size: str = "small", seed: int = 1, device="cuda", n_vocab: int = N_VOCAB,
                 n_ctx: int = N_TEXT_CTX, prompt=SOT_SEQUENCE, eot: int = EOT):
        self.device = torch.device(device)
        self.size = size
        d, L, H = SIZES[size]
        self.d, self.layers_n, self.heads = d, L, H
        self.n_vocab, self.n_ctx = n_vocab, n_ctx
        self.prompt = tuple(int(t) for t in prompt)
        self.eot = int(eot)
        if not 1 <= len(self.prompt) < n_ctx:
            raise ValueError("prompt must hold 1 .. n_ctx-1 tokens")
        g = torch.Generator().manual_seed(seed)
        dev = self.device

        def rnd(*shape, fan_in):
            return torch.randn(*shape, generator=g) / math.sqrt(fan_in)

        def small(n):
            return 0.02 * torch.randn(n, generator=g)

        def ln():
            return ((1.0 + 0.1 * torch.randn(d, generator=g)).to(dev), small(d).to(dev))

        emb = 0.1 * torch.randn(n_vocab, d, generator=g)
        self.tok_emb = emb.to(dev, torch.bfloat16)
        self.pos_emb = (0.02 * torch.randn(n_ctx, d, generator=g)).to(dev, torch.bfloat16)
        self.blocks = []
        for _ in range(L):
            bqkv = torch.cat([small(d), torch.zeros(d), small(d)])       # key projection: no bias
            bkv = torch.cat([torch.zeros(d), small(d)])
            self.blocks.append(DecoderBlock(
                ln(), TR.make_fp8_linear(rnd(3 * d, d, fan_in=d), bqkv, dev),
                TR.make_fp8_linear(rnd(d, d, fan_in=d), small(d), dev),
                ln(), TR.make_fp8_linear(rnd(d, d, fan_in=d), small(d), dev),
                TR.make_fp8_linear(rnd(2 * d, d, fan_in=d), bkv, dev),
                TR.make_fp8_linear(rnd(d, d, fan_in=d), small(d), dev),
                ln(), TR.make_fp8_linear(rnd(4 * d, d, fan_in=d), small(4 * d), dev),
                TR.make_fp8_linear(rnd(d, 4 * d, fan_in=4 * d), small(d), dev)))
        self.ln_final = ln()
        self._make_logit_weight()
        self._ws: dict = {}
        self._graphs: dict = {}
        self._geom = None
        self.ws_tag = ""             # workspace key prefix (one decode state per frame lane)
        self.fused_linear = True     # dec_linear_kernel (LN/quantise fused) where K <= 3072

    def _make_logit_weight(self):
        """Logits use the token embedding (tied), quantised to e4m3 per vocabulary row; rows are
        padded to a multiple of 128 (zero weights, never selected: the argmax scans n_vocab)."""
        vp = -(-self.n_vocab // 128) * 128
        w = torch.zeros(vp, self.d)
        w[:self.n_vocab] = self.tok_emb.float().cpu()
        self.logits = TR.make_fp8_linear(w, None, self.device)

    # ---- weights ---------------------------------------------------------------------------------
    def named_layers(self):
        yield "tok_emb", self.tok_emb
        yield "pos_emb", self.pos_emb
        for i, b in enumerate(self.blocks):
            for name in ("ln1", "qkv", "out", "lnx", "cq", "ckv", "cout", "ln2", "fc1", "fc2"):
                yield f"blocks.{i}.{name}", getattr(b, name)
        yield "ln_final", self.ln_final
        yield "logits", self.logits

    def config(self) -> dict:
        return {"size": self.size, "n_vocab": self.n_vocab, "n_ctx": self.n_ctx,
                "prompt": list(self.prompt), "eot": self.eot}

    def _weights_loaded(self):
        self._graphs.clear()

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
        self._graphs.clear()
        self._geom = None

    @staticmethod
    def _rows(features: torch.Tensor):
        """Encoder features [B, T, d] -> (rows [B*S, d], S): zero-copy when the batch stride is a
        whole number of rows (the encoder's padded [B, T+1, d] output), else a packed copy."""
        B, T, d = features.shape
        if features.stride(2) == 1 and features.stride(1) == d and features.stride(0) % d == 0:
            S = features.stride(0) // d
            if features.storage_offset() + B * S * d <= features.untyped_storage().nbytes() // features.element_size():
                return torch.as_strided(features, (B * S, d), (d, 1)), S
        return features.contiguous().view(B * T, d), T

    def prepare(self, features: torch.Tensor):
        """Cross-attention K/V for a batch of encoder outputs; resets the decode state to the
        prompt's first token at position 0."""
        B, T, d = features.shape
        if d != self.d:
            raise ValueError(f"features width {d} != decoder width {self.d}")
        rows, S = self._rows(features.to(torch.bfloat16) if features.dtype != torch.bfloat16 else features)
        self._geom = (B, T, S)
        q8 = self._buf("enc_q8", (B * S, d), torch.uint8)
        s8 = self._buf("enc_s8", (B * S,), torch.float32)
        TR.rownorm(rows, q=q8, qs=s8)
        for i, blk in enumerate(self.blocks):
            TR.linear_fp8(q8, s8, blk.ckv, out=self._buf(f"kv_cross{i}", (B * S, 2 * d)))
        self.reset(B)

    def reset(self, B: int):
        st = self._state(B)
        st["ids"].fill_(self.prompt[0])
        st["pos"].zero_()
        st["done"].zero_()
        st["counter"].zero_()
        st["tokens"].fill_(self.eot)
        st["tokens"][:, 0] = self.prompt[0]

    def _state(self, B):
        return {"ids": self._buf("ids", (B,), torch.int32), "pos": self._buf("pos", (1,), torch.int32),
                "done": self._buf("done", (B,), torch.int32),
                "counter": self._buf("counter", (1,), torch.int32),
                "tokens": self._buf("tokens", (B, self.n_ctx), torch.int32),
                "forced": self._buf(f"forced{len(self.prompt)}", (len(self.prompt),), torch.int32)}

    def step(self):
        """One token for every sequence (graph-capturable: no host reads, no allocation)."""
        B, T, S = self._geom
        d, H, n_ctx = self.d, self.heads, self.n_ctx
        st = self._state(B)
        x = self._buf("x", (B, d))
        q8 = self._buf("q8", (B, 4 * d), torch.uint8)
        s8 = self._buf("s8", (B,), torch.float32)
        qkv = self._buf("qkv", (B, 3 * d))
        att = self._buf("att", (B, d))
        cq = self._buf("cq", (B, d))
        h = self._buf("h", (B, 4 * d))
        logits = self._buf("logits", (B, self.logits.n))
        work = self._buf("work", (attn_decode_work(B, H, max(n_ctx, T)),), torch.float32)
        scale = (d // H) ** -0.5
        qd = q8[:, :d]

        def lin(src, layer, out, ln=None, residual=None, act=TR.ACT_NONE):
            if self.fused_linear and src.shape[1] <= 3072:
                return dec_linear(src, layer, out, ln, residual, act)
            qs = q8[:, :src.shape[1]]
            TR.rownorm(src, *(ln or (None, None)), q=qs, qs=s8)
            return TR.linear_fp8(qs, s8, layer, out=out, residual=residual, act=act)

        torch.ops.aiko.embed_tokens_out(st["ids"], st["pos"], self.tok_emb, self.pos_emb, x)
        for i, blk in enumerate(self.blocks):
            kvs = self._buf(f"kv_self{i}", (B * n_ctx, 2 * d))
            kvc = self._buf(f"kv_cross{i}", (B * S, 2 * d))
            lin(x, blk.qkv, qkv, ln=blk.ln1)
            attn_decode(qkv[:, :d], kvs[:, :d], kvs[:, d:], att, B, H, n_ctx, 0, scale, work,
                        pos=st["pos"], knew=qkv[:, d:2 * d], vnew=qkv[:, 2 * d:])
            lin(att, blk.out, x, residual=x)
            lin(x, blk.cq, cq, ln=blk.lnx)
            attn_decode(cq, kvc[:, :d], kvc[:, d:], att, B, H, S, T, scale, work)
            lin(att, blk.cout, x, residual=x)
            lin(x, blk.fc1, h, ln=blk.ln2, act=TR.ACT_GELU)
            lin(h, blk.fc2, x, residual=x)
        lin(x, self.logits, logits, ln=self.ln_final)
        torch.ops.aiko.argmax_step_out(logits, self.n_vocab, st["ids"], st["pos"], st["tokens"],
                                       st["forced"], self.eot, st["done"], st["counter"])
        return logits

    def _replay_step(self, use_graph: bool):
        if not use_graph or self.device.type != "cuda":
            self.step()
            return
        key = (self.ws_tag,) + self._geom
        g = self._graphs.get(key)
        if g is None:
            # warm-up (tile selection, workspace allocation) runs eagerly on a scratch state
            st = self._state(self._geom[0])
            saved = {k: v.clone() for k, v in st.items()}
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self.step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.step()
            for k, v in st.items():                 # capture ran nothing; undo the warm-up
                v.copy_(saved[k])
            self._graphs[key] = g
        g.replay()

    def transcribe(self, features: torch.Tensor, max_new_tokens: int = 96, use_graph: bool = True,
                   check_every: int = 8) -> torch.Tensor:
        """Greedy decoding after the prompt; returns int32 [B, n] on the device (prompt first,
        ``eot`` after each sequence's end)."""
        self.prepare(features)
        B = features.shape[0]
        st = self._state(B)
        st["forced"].copy_(torch.tensor(self.prompt, dtype=torch.int32))
        n_steps = min(len(self.prompt) - 1 + max_new_tokens, self.n_ctx - 1)
        for s in range(n_steps):
            self._replay_step(use_graph)
            if check_every and s >= len(self.prompt) and (s + 1) % check_every == 0 and bool(st["done"].all()):
                n_steps = s + 1
                break
        return st["tokens"][:, :n_steps + 1]

    # ---- fp32 torch reference (tests only): same (fp8-dequantised) weights, teacher forced ------
    def reference_logits(self, features: torch.Tensor, tokens: torch.Tensor) -> torch.Tensor:
        """fp32 logits [B, n, n_vocab] for ``tokens`` [B, n] given encoder ``features``."""
        import torch.nn.functional as F
        d, H = self.d, self.heads
        B, n = tokens.shape
        enc = features.float()
        tok = self.tok_emb.float()
        x = tok[tokens.long()] + self.pos_emb.float()[:n]

        def lin(t, layer):
            y = t @ layer.ref_weight.T.to(t.device)
            return y if layer.bias is None else y + layer.bias

        def heads(t):
            return t.view(B, t.shape[1], H, d // H).transpose(1, 2)

        for blk in self.blocks:
            h = F.layer_norm(x, (d,), blk.ln1[0], blk.ln1[1], 1e-5)
            q, k, v = lin(h, blk.qkv).split(d, dim=-1)
            a = F.scaled_dot_product_attention(heads(q), heads(k), heads(v), is_causal=True)
            x = x + lin(a.transpose(1, 2).reshape(B, n, d), blk.out)
            h = F.layer_norm(x, (d,), blk.lnx[0], blk.lnx[1], 1e-5)
            q = lin(h, blk.cq)
            k, v = lin(enc, blk.ckv).split(d, dim=-1)
            a = F.scaled_dot_product_attention(heads(q), heads(k), heads(v))
            x = x + lin(a.transpose(1, 2).reshape(B, n, d), blk.cout)
            h = F.layer_norm(x, (d,), blk.ln2[0], blk.ln2[1], 1e-5)
            x = x + lin(F.gelu(lin(h, blk.fc1)), blk.fc2)
        x = F.layer_norm(x, (d,), self.ln_final[0], self.ln_final[1], 1e-5)
        return (x @ self.logits.ref_weight.T.to(x.device))[..., :self.n_vocab]


def decode_text(tokens, tokenizer=None, eot: int = EOT, skip_below: int = EOT) -> list[str]:
    """Token ids -> strings.  ``tokenizer`` is a ``tokenizers.Tokenizer`` (e.g. loaded from a
    Whisper ``tokenizer.json``); without one, ids are rendered as ``<id>`` (no vocabulary files
    ship offline).  Special tokens (>= ``skip_below``) and everything after ``eot`` are dropped."""
    rows = tokens.tolist() if hasattr(tokens, "tolist") else tokens
    out = []
    for row in rows:
        ids = []
        for t in row:
            if t == eot:
                break
            if t < skip_below:
                ids.append(int(t))
        if tokenizer is not None:
            out.append(tokenizer.decode(ids).strip())
        else:
            out.append(" ".join(f"<{t}>" for t in ids))
    return out
