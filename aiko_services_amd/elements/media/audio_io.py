"""Audio elements.

The reference's live audio code is a skeleton (``elements/media/audio_io.py:76-159``) plus a
large dead docstring (``:162-642``: filter, resampler, FFT, microphone, speaker, remote
send/receive) and the speech example's ``PE_AudioFraming`` (``examples/speech/
speech_elements.py:60-83``).  This module implements the working subset without device
audio libraries: WAV read/write (stdlib ``wave``), chunking, sliding-window framing,
resampling, FFT, and a synthetic chunk source for the streamed Whisper-encoder config.
Audio flows as float32 mono numpy arrays (or device tensors on the GPU path).
"""
from __future__ import annotations

import wave
from collections import deque
from pathlib import Path

import numpy as np

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from .common_io import DataSource, DataTarget

__all__ = ["AudioOutput", "AudioReadFile", "AudioWriteFile", "AudioFraming", "AudioResampler",
           "PE_FFT", "AudioSynthetic", "read_wav", "write_wav"]


def read_wav(path):
    with wave.open(str(path), "rb") as w:
        rate, ch, width, n = w.getframerate(), w.getnchannels(), w.getsampwidth(), w.getnframes()
        raw = w.readframes(n)
    dtype = {1: np.uint8, 2: np.int16, 4: np.int32}[width]
    x = np.frombuffer(raw, dtype).astype(np.float32)
    if width == 1:
        x = (x - 128.0) / 128.0
    else:
        x /= float(2 ** (8 * width - 1))
    if ch > 1:
        x = x.reshape(-1, ch).mean(axis=1)
    return x, rate


def write_wav(path, samples, rate=16000):
    x = np.clip(np.asarray(samples, np.float32), -1.0, 1.0)
    with wave.open(str(path), "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(rate))
        w.writeframes((x * 32767.0).astype(np.int16).tobytes())


def resample_linear(x, rate_in, rate_out):
    if rate_in == rate_out:
        return x
    n_out = int(round(len(x) * rate_out / rate_in))
    t = np.arange(n_out, dtype=np.float64) * (rate_in / rate_out)
    return np.interp(t, np.arange(len(x)), x).astype(np.float32)


class AudioOutput(PipelineElement):
    def __init__(self, context):
        context.set_protocol("audio_output:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, audio_samples):
        return StreamEvent.OKAY, {"audio_samples": audio_samples}


class AudioReadFile(DataSource):
    """WAV files -> chunks of ``chunk_duration`` s (default 5 s) at ``sample_rate`` (16 kHz)."""

    def __init__(self, context):
        context.set_protocol("audio_read_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        stream.variables["audio_chunks"] = None
        return super().start_stream(stream, stream_id, use_create_frame=False)

    def _chunks(self, path):
        rate_out, _ = self.get_parameter("sample_rate", 16000)
        dur, _ = self.get_parameter("chunk_duration", 5.0)
        x, rate = read_wav(path)
        x = resample_linear(x, rate, int(rate_out))
        n = int(float(dur) * int(rate_out))
        for i in range(0, len(x), n):
            c = x[i:i + n]
            if len(c) < n:
                c = np.pad(c, (0, n - len(c)))
            yield c

    def frame_generator(self, stream, frame_id):
        gen = stream.variables.get("audio_chunks")
        while True:
            if gen is None:
                try:
                    path, _ = next(stream.variables["source_paths_generator"])
                except StopIteration:
                    return StreamEvent.STOP, {"diagnostic": "End of audio file(s)"}
                try:
                    gen = self._chunks(path)
                except (wave.Error, EOFError, KeyError) as exc:
                    return StreamEvent.ERROR, {"diagnostic": f"Couldn't open audio file {path}: {exc}"}
                stream.variables["audio_chunks"] = gen
            try:
                return StreamEvent.OKAY, {"audio_samples": next(gen)}
            except StopIteration:
                gen = None
                stream.variables["audio_chunks"] = None

    def process_frame(self, stream, audio_samples):
        return StreamEvent.OKAY, {"audio_samples": audio_samples}


class AudioWriteFile(DataTarget):
    def __init__(self, context):
        context.set_protocol("audio_write_file:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, audio_samples):
        rate, _ = self.get_parameter("sample_rate", 16000)
        path = self.next_target_path(stream)
        try:
            write_wav(path, np.asarray(audio_samples), int(rate))
        except Exception as exc:
            return StreamEvent.ERROR, {"diagnostic": f"Error saving audio: {exc}"}
        return StreamEvent.OKAY, {}


class AudioFraming(PipelineElement):
    """Sliding window of the last ``window_chunks`` chunks (speech example's PE_AudioFraming)."""

    def __init__(self, context):
        context.set_protocol("audio_framing:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        n, _ = self.get_parameter("window_chunks", 2)
        stream.variables["audio_window"] = deque(maxlen=int(n))
        return StreamEvent.OKAY, {}

    def process_frame(self, stream, audio_samples):
        window = stream.variables.setdefault("audio_window", deque(maxlen=2))
        window.append(np.asarray(audio_samples, np.float32))
        return StreamEvent.OKAY, {"audio_samples": np.concatenate(list(window))}


class AudioResampler(PipelineElement):
    def __init__(self, context):
        context.set_protocol("audio_resampler:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, audio_samples):
        rin, _ = self.get_parameter("sample_rate_in", 48000)
        rout, _ = self.get_parameter("sample_rate_out", 16000)
        return StreamEvent.OKAY, {"audio_samples": resample_linear(np.asarray(audio_samples, np.float32),
                                                                   int(rin), int(rout))}


class PE_FFT(PipelineElement):
    """Magnitude spectrum of each chunk (reference dead ``PE_FFT``)."""

    def __init__(self, context):
        context.set_protocol("fft:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, audio_samples):
        x = np.asarray(audio_samples, np.float32)
        spectrum = np.abs(np.fft.rfft(x))
        rate, _ = self.get_parameter("sample_rate", 16000)
        freqs = np.fft.rfftfreq(len(x), 1.0 / int(rate))
        return StreamEvent.OKAY, {"amplitudes": spectrum, "frequencies": freqs}


class AudioSynthetic(PipelineElement):
    """Synthetic 16 kHz chunks (sine sweep + noise): the streamed-audio source of config 5."""

    def __init__(self, context):
        context.set_protocol("audio_synthetic:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        frames, _ = self.get_parameter("frames", 0)
        stream.variables["audio_frames_left"] = int(frames) if frames else None
        rate, _ = self.get_parameter("rate", None)
        self.create_frames(stream, self.frame_generator, rate=float(rate) if rate else None)
        return StreamEvent.OKAY, {}

    def frame_generator(self, stream, frame_id):
        left = stream.variables.get("audio_frames_left")
        if left is not None:
            if left <= 0:
                return StreamEvent.STOP, {"diagnostic": "All frames generated"}
            stream.variables["audio_frames_left"] = left - 1
        sr, _ = self.get_parameter("sample_rate", 16000)
        dur, _ = self.get_parameter("chunk_duration", 5.0)
        n = int(int(sr) * float(dur))
        t = (np.arange(n) + frame_id * n) / float(sr)
        rng = np.random.default_rng(frame_id)
        x = 0.3 * np.sin(2 * np.pi * (220 + 30 * np.sin(t)) * t) + 0.05 * rng.standard_normal(n)
        return StreamEvent.OKAY, {"audio_samples": x.astype(np.float32)}

    def process_frame(self, stream, audio_samples):
        return StreamEvent.OKAY, {"audio_samples": audio_samples}
