"""Audio front end ops (``csrc/kernels/audio_ops.hip``): Whisper log-mel spectrogram.

``mel_filters`` builds the Slaney-style mel filterbank (the librosa default Whisper ships as
``mel_filters.npz``; computed here since no assets are available offline)."""
from __future__ import annotations

import math

import torch

SAMPLE_RATE = 16000
N_FFT = 400
HOP = 160

__all__ = ["mel_filters", "log_mel", "log_mel_ref", "SAMPLE_RATE", "N_FFT", "HOP"]


def _hz_to_mel(f):
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return f / f_sp if f < min_log_hz else min_log_mel + math.log(f / min_log_hz) / logstep


def _mel_to_hz(m: torch.Tensor) -> torch.Tensor:
    f_sp, min_log_hz = 200.0 / 3, 1000.0
    min_log_mel, logstep = min_log_hz / f_sp, math.log(6.4) / 27.0
    return torch.where(m >= min_log_mel, min_log_hz * torch.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filters(n_mels: int = 80, n_fft: int = N_FFT, sr: int = SAMPLE_RATE) -> torch.Tensor:
    """[n_mels, n_fft // 2 + 1] fp32 Slaney mel filterbank (area-normalised triangles)."""
    fft_freqs = torch.linspace(0, sr / 2, n_fft // 2 + 1, dtype=torch.float64)
    mels = torch.linspace(_hz_to_mel(0.0), _hz_to_mel(sr / 2), n_mels + 2, dtype=torch.float64)
    mel_f = _mel_to_hz(mels)
    fdiff = mel_f[1:] - mel_f[:-1]
    ramps = mel_f[:, None] - fft_freqs[None, :]
    w = torch.zeros(n_mels, n_fft // 2 + 1, dtype=torch.float64)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = torch.clamp(torch.minimum(lower, upper), min=0)
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    return (w * enorm[:, None]).float()


_RANGES: dict = {}


def mel_ranges(filters: torch.Tensor) -> torch.Tensor:
    """int32 [n_mels, 3] = (first nonzero bin, run length, offset into the packed weights) of
    each triangular filter — the log-mel kernel's sparse filterbank (cached per tensor)."""
    key = (filters.data_ptr(), filters._version, tuple(filters.shape))
    r = _RANGES.get(key)
    if r is None:
        rows, off = [], 0
        for w in filters.detach().float().cpu():
            nz = torch.nonzero(w != 0).flatten()
            lo = int(nz[0]) if nz.numel() else 0
            n = int(nz[-1]) - lo + 1 if nz.numel() else 0
            rows.append((lo, n, off))
            off += n
        if off > 2048:
            raise ValueError(f"mel filterbank has {off} nonzero span elements (kernel limit 2048)")
        r = _RANGES[key] = torch.tensor(rows, dtype=torch.int32, device=filters.device)
    return r


def log_mel(audio: torch.Tensor, filters: torch.Tensor, out: torch.Tensor, rows: int, pad: int,
            work: torch.Tensor | None = None, gmax: torch.Tensor | None = None, frames: int | None = None):
    """fp32 audio [B, N] -> Whisper-normalised log-mel, bf16, frame t of clip b at row
    ``b*rows + pad + t`` of ``out`` [B*rows, n_mels] (other rows zero: conv padding)."""
    B, N = audio.shape
    F = frames if frames is not None else N // HOP
    n_mels = filters.shape[0]
    if work is None:
        work = torch.empty(B * F * n_mels, dtype=torch.float32, device=audio.device)
    if gmax is None:
        gmax = torch.empty(B, dtype=torch.int32, device=audio.device)
    torch.ops.aiko.logmel_out(audio, filters, mel_ranges(filters), N_FFT, HOP, F, work, gmax, out, rows, pad)
    return out


def log_mel_ref(audio: torch.Tensor, filters: torch.Tensor, frames: int | None = None) -> torch.Tensor:
    """Whisper's reference log-mel (torch.stft), fp32 [B, n_mels, F]."""
    window = torch.hann_window(N_FFT, device=audio.device)
    stft = torch.stft(audio, N_FFT, HOP, window=window, return_complex=True)
    mag = stft[..., :-1].abs() ** 2
    if frames is not None:
        mag = mag[..., :frames]
    mel = filters.to(audio.device) @ mag
    log_spec = torch.clamp(mel, min=1e-10).log10()
    log_spec = torch.maximum(log_spec, log_spec.amax(dim=(1, 2), keepdim=True) - 8.0)
    return (log_spec + 4.0) / 4.0


def window_shift(src: torch.Tensor, chunk: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """``dst[b] = concat(src[b, n:], chunk[b])`` — a sliding audio window advanced by one chunk
    (fp32 [B, W] / [B, n]); one HIP kernel on the GPU, torch slicing on the CPU."""
    n = chunk.shape[1]
    if dst.is_cuda:
        torch.ops.aiko.window_shift_out(src, chunk, dst)
    else:
        dst[:, :dst.shape[1] - n].copy_(src[:, n:])
        dst[:, dst.shape[1] - n:].copy_(chunk)
    return dst
