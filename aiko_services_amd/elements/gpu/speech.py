"""GPU speech PipelineElements — BASELINE config 5, Whisper encoder on streamed audio chunks.

    "(AudioChunks AudioWindow WhisperEncoder FeatureSink)"

* ``AudioChunks``   — ``streams`` concurrent audio streams, each producing a ``chunk``-second
  16 kHz chunk per frame directly in HBM (synthetic: tones + noise from a rotating pool), or
  uploads host chunks (numpy / CPU tensors from ``AudioReadFile`` / ``AudioSynthetic``) through
  pinned staging buffers;
* ``AudioWindow``   — per-stream sliding window of the last ``window`` seconds kept on the GPU
  (the reference's ``PE_AudioFraming`` LRU of chunks, ``examples/speech/speech_elements.py:
  60-83``, as one device ring per stream: shift + append, no host copies);
* ``WhisperEncoder`` — log-mel + Whisper encoder (fp8 linear layers) over the windows,
  optional hipGraph capture; emits encoder features [B, T, d] on the device;
* ``FeatureSink``   — mean-pooled features to pinned host memory as a DeviceResult (the
  encoder-only BASELINE config's consumer);
* ``WhisperTranscribe`` — greedy text decoding of the features (``models/whisper_decoder.py``),
  ``{"tokens", "text"}`` like the reference's ``PE_WhisperX`` output;
* ``SpeechToText``  — ``PE_WhisperX`` in one element: audio -> encoder -> decoder -> text.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ...gpu.element import DeviceResult, GpuPipelineElement, HostRing
from ...pipeline.stream import StreamEvent

__all__ = ["AudioChunks", "AudioWindow", "WhisperEncoder", "WhisperTranscribe", "SpeechToText", "FeatureSink"]

RATE = 16000


def _p(el, name, default):
    return el.get_parameter(name, default)[0]


class AudioChunks(GpuPipelineElement):
    lane_safe = True          # read-only synthetic pool; pinned upload ring

    def __init__(self, context):
        context.set_protocol("audio_chunks:0")
        super().__init__(context)
        self._pool = None
        self._cursor = 0
        self._pinned: list = []
        self._pin_slot = 0

    def _synthetic(self):
        if self._pool is None:
            B = int(_p(self, "streams", 8))
            n = int(float(_p(self, "chunk", 5.0)) * RATE)
            g = torch.Generator(device=self.device).manual_seed(int(_p(self, "seed", 0)))
            t = torch.arange(n, device=self.device, dtype=torch.float32) / RATE
            self._pool = []
            for _ in range(int(_p(self, "pool", 4))):
                f = 100 + 900 * torch.rand(B, 1, device=self.device, generator=g)
                noise = 0.02 * torch.randn(B, n, device=self.device, generator=g)
                self._pool.append((0.3 * torch.sin(2 * torch.pi * f * t) + noise).contiguous())
        x = self._pool[self._cursor % len(self._pool)]
        self._cursor += 1
        return x

    def _upload(self, audio):
        x = torch.as_tensor(np.asarray(audio, dtype=np.float32)) if not isinstance(audio, torch.Tensor) else audio
        if x.dim() == 1:
            x = x[None]
        if x.device.type == "cuda":
            return x.float()
        if not self._pinned or self._pinned[0][0].shape != x.shape:
            self._pinned = [[torch.empty(x.shape, dtype=torch.float32, pin_memory=True), None]
                            for _ in range(4)]
        slot = self._pinned[self._pin_slot]
        self._pin_slot = (self._pin_slot + 1) % len(self._pinned)
        if slot[1] is not None:
            slot[1].synchronize()          # the H2D copy that last read this slot is done
        slot[0].copy_(x)
        out = slot[0].to(self.device, non_blocking=True)
        slot[1] = torch.cuda.Event()
        slot[1].record()
        return out

    def process_frame(self, stream, audio_samples=None, **kwargs):
        audio = self._synthetic() if audio_samples is None else self._upload(audio_samples)
        return StreamEvent.OKAY, {"audio": audio, "t_submit": time.perf_counter()}


class AudioWindow(GpuPipelineElement):
    """Per-stream sliding window over the last ``window`` seconds: frame k writes ring slot
    k % R from slot (k-1) % R.  With L frame lanes, R = L + 1 and every update waits for the
    previous frame's update (an event chain across the lane streams): slot k % R was last
    read by frame k-L's window update and by the encoder of frame k-R, which ran on frame
    k-1's lane before frame k-1's update — so the chain orders every reuse."""
    lane_safe = True

    def __init__(self, context):
        context.set_protocol("audio_window:0")
        super().__init__(context)
        self.window = int(float(_p(self, "window", 30.0)) * RATE)
        self._ring = None
        self._last = None

    def process_frame(self, stream, audio):
        B, n = audio.shape
        W = self.window
        lanes = getattr(self.pipeline, "_lanes_cfg", (1, None))[0] if self.pipeline is not None else 1
        R = max(2, lanes + 1)
        if self._ring is None or self._ring[0].shape[0] != B or len(self._ring) != R:
            self._ring = [torch.zeros(B, W, dtype=torch.float32, device=self.device) for _ in range(R)]
            self._cur = 0
            self._last = None
        src = self._ring[self._cur]
        self._cur = (self._cur + 1) % R
        dst = self._ring[self._cur]
        if self._last is not None and self.device.type == "cuda":
            torch.cuda.current_stream(self.device).wait_event(self._last)
        if n >= W:
            dst.copy_(audio[:, n - W:])
        else:
            from ...ops.audio import window_shift
            window_shift(src, audio.contiguous(), dst)     # one aiko:: kernel on the GPU
        if self.device.type == "cuda":
            self._last = torch.cuda.Event()
            self._last.record()
        return StreamEvent.OKAY, {"audio": dst}


class WhisperEncoder(GpuPipelineElement):
    lane_safe = True          # one model workspace per lane

    def __init__(self, context):
        context.set_protocol("whisper_encoder:0")
        super().__init__(context)
        from ...models.whisper import WhisperEncoder as Model
        from ...ops import require_native
        require_native()
        self.model = Model(size=str(_p(self, "size", "small")), seed=int(_p(self, "seed", 0)),
                           device=self.device)
        self.load_model_weights(self.model)
        self._tuned = set()

    def _run(self, audio):
        self.model.ws_tag = f"lane{self.lane}." if self.lane else ""
        return self.model.encode(audio)

    def process_frame(self, stream, audio):
        key = (tuple(audio.shape),)
        if key not in self._tuned:
            from ...ops import conv as C
            if str(_p(self, "autotune", self.gpu_config.autotune)).lower() in ("true", "1", "yes"):
                with C.autotune():
                    self._run(audio)
            else:
                self._run(audio)
            self._tuned.add(key)
        return StreamEvent.OKAY, {"features": self.run_maybe_captured(key, self._run, audio)}


_SILENCE = ("", "you", "thank you.", "thanks for watching!")


def _load_tokenizer(el):
    """Optional ``tokenizer`` parameter: a Whisper ``tokenizer.json`` read with the
    ``tokenizers`` library (no vocabulary ships offline; without it ids render as ``<id>``)."""
    path, found = el.get_parameter("tokenizer")
    if not found or not path:
        return None
    from tokenizers import Tokenizer
    return Tokenizer.from_file(str(path))


def _reply(text: str) -> str:
    """The reference's post-filter (``speech_elements.py:240-255``): lower-case, strip a final
    full stop, map Whisper's usual hallucinations on silence to ``<silence>``."""
    t = text.strip().lower()
    if t in _SILENCE:
        return "<silence>"
    return t.removesuffix(".")


class WhisperTranscribe(GpuPipelineElement):
    """Greedy Whisper decoding of encoder ``features`` [B, T, d] -> ``tokens`` (int32 [B, n] on
    the host) and ``text`` (one string per stream, "<silence>" when empty).  Parameters:
    ``size``, ``seed``, ``max_tokens`` (default 96), ``tokenizer`` (tokenizer.json path),
    ``weights``, ``graph`` (hipGraph-replayed decode steps, default on), ``stop_early``
    (default on: stop once every stream has emitted end-of-text, checked every 8 steps),
    ``defer_text`` (default off: with it the tokens come back as a DeviceResult on pinned host
    memory without a host synchronisation and ``text`` is not produced — for throughput runs
    where the next frame's encoder should queue behind this frame's decoder)."""
    lane_safe = True          # one decode state / graph per lane (ws_tag)

    def __init__(self, context):
        context.set_protocol("speech_to_text:0")
        super().__init__(context)
        from ...models.whisper_decoder import WhisperDecoder
        from ...ops import require_native
        require_native()
        self.model = WhisperDecoder(size=str(_p(self, "size", "small")), seed=int(_p(self, "seed", 1)),
                                    device=self.device)
        self.load_model_weights(self.model)
        self.tokenizer = _load_tokenizer(self)

    def _decode(self, features, stop: bool):
        self.model.ws_tag = f"lane{self.lane}." if self.lane else ""
        return self.model.transcribe(features, max_new_tokens=int(_p(self, "max_tokens", 96)),
                                     use_graph=self.use_graph, check_every=8 if stop else 0)

    def transcribe(self, features):
        from ...models.whisper_decoder import decode_text
        stop = str(_p(self, "stop_early", True)).lower() in ("true", "1", "yes")
        tokens = self._decode(features, stop).cpu()
        texts = [_reply(t) for t in decode_text(tokens, self.tokenizer, eot=self.model.eot)]
        return tokens, texts

    def process_frame(self, stream, features, t_submit=None):
        t0 = t_submit if isinstance(t_submit, float) else None
        if str(_p(self, "defer_text", False)).lower() in ("true", "1", "yes"):
            tok = self._decode(features, False)
            key = (tuple(tok.shape), self.lane)
            bufs = self.__dict__.setdefault("_pinned", {})
            ring = bufs.get(key)
            if ring is None:
                ring = bufs[key] = [[torch.empty(tok.shape, dtype=tok.dtype, pin_memory=True), None]
                                    for _ in range(4)]
            slot = ring[0]
            ring.append(ring.pop(0))
            if slot[1] is not None:
                slot[1].synchronize()          # this slot's previous copy has landed
            slot[0].copy_(tok, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            slot[1] = ev
            return StreamEvent.OKAY, {"transcript": DeviceResult({"tokens": slot[0]}, ev, t_submit=t0)}
        tokens, texts = self.transcribe(features)
        return StreamEvent.OKAY, {"tokens": tokens, "text": texts[0] if len(texts) == 1 else texts,
                                  "transcript": DeviceResult({"tokens": tokens}, None, t_submit=t0)}


class SpeechToText(WhisperTranscribe):
    """The reference's ``PE_WhisperX`` shape in one element: ``audio`` (16 kHz samples, [N] or
    [B, N], host or device) -> log-mel + encoder + greedy decoder -> ``{"text": ...}``."""

    def __init__(self, context):
        super().__init__(context)
        from ...models.whisper import WhisperEncoder as Encoder
        self.encoder = Encoder(size=str(_p(self, "size", "small")), seed=int(_p(self, "encoder_seed", 0)),
                               device=self.device)
        path, found = self.get_parameter("encoder_weights")
        if found and path:
            self.encoder.load(str(path))

    def process_frame(self, stream, audio):
        x = audio if isinstance(audio, torch.Tensor) else torch.as_tensor(np.asarray(audio, dtype=np.float32))
        x = x.to(self.device, torch.float32)
        if x.dim() == 1:
            x = x[None]
        n = x.shape[1] - x.shape[1] % 320                     # whole encoder frames (320 samples)
        if n <= 0:
            return StreamEvent.OKAY, {"text": "<silence>", "tokens": None}
        tokens, texts = self.transcribe(self.encoder.encode(x[:, :n].contiguous()))
        return StreamEvent.OKAY, {"tokens": tokens, "text": texts[0] if len(texts) == 1 else texts}


class FeatureSink(GpuPipelineElement):
    lane_safe = True          # device + pinned buffers per lane

    def __init__(self, context):
        context.set_protocol("feature_sink:0")
        super().__init__(context)
        self._bufs: dict = {}

    def process_frame(self, stream, features, t_submit=None):
        B, T, d = features.shape
        b = self._bufs.get((B, d, self.lane))
        if b is None:
            pin = self.device.type == "cuda"
            b = self._bufs[(B, d, self.lane)] = {
                "pooled": torch.empty(B, d, dtype=torch.float32, device=self.device),
                "host": HostRing(lambda: torch.empty(B, d, dtype=torch.float32, pin_memory=pin), 8)}
        if self.device.type == "cuda":
            from ...ops.vision import mean_rows
            mean_rows(features, out=b["pooled"])     # HIP reduction kernel (reads the T-prefix view)
        else:
            torch.mean(features, dim=1, dtype=torch.float32, out=b["pooled"])
        slot, h = b["host"].acquire()
        h.copy_(b["pooled"], non_blocking=True)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        result = DeviceResult({"pooled": h}, ev, t_submit=t_submit if isinstance(t_submit, float) else None)
        return StreamEvent.OKAY, {"embedding": b["host"].bind(slot, result)}
