"""Audio elements.

The reference's live audio code is a skeleton (``elements/media/audio_io.py:76-159``) plus a
large dead docstring (``:162-642``: filter, resampler, FFT, XY graph, microphone, speaker,
remote send/receive) and the speech example's ``PE_AudioFraming`` (``examples/speech/
speech_elements.py:60-83``).  This module implements all of them: WAV read/write (stdlib
``wave``), chunking, sliding-window framing, resampling, FFT, spectrum filter and band
consolidation, an XY-graph renderer (numpy raster instead of pygal + cv2 window), remote
send/receive of arrays over binary MQTT topics (``zlib(np.save)`` as in the reference, but
never pickled), and a synthetic chunk source for the streamed Whisper-encoder config.
Microphone / speaker elements need ``sounddevice`` or ``pyaudio``; neither is installed in
this image, so they raise a clear error when constructed without one.
Audio flows as float32 mono numpy arrays (or device tensors on the GPU path).
"""
from __future__ import annotations

import threading
import time
import wave
import zlib
from collections import deque
from io import BytesIO
from pathlib import Path

import numpy as np

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from .common_io import DataSource, DataTarget

__all__ = ["AudioOutput", "AudioReadFile", "AudioWriteFile", "AudioFraming", "AudioResampler",
           "PE_FFT", "AudioSynthetic", "PE_AudioFilter", "PE_AudioResampler", "PE_GraphXY",
           "PE_MicrophonePA", "PE_MicrophoneSD", "PE_Speaker", "PE_RemoteSend0", "PE_RemoteSend1",
           "PE_RemoteSend2", "PE_RemoteReceive0", "PE_RemoteReceive1", "PE_RemoteReceive2",
           "encode_array", "decode_array", "read_wav", "write_wav"]


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


# ---- spectrum post-processing (reference dead PE_AudioFilter / PE_AudioResampler / PE_GraphXY) --

class PE_AudioFilter(PipelineElement):
    """Keep the loudest ``samples_maximum`` spectrum points inside the amplitude / frequency box
    (reference ``audio_io.py`` dead ``PE_AudioFilter``; the limits are parameters here)."""

    def __init__(self, context):
        context.set_protocol("audio_filter:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, amplitudes, frequencies):
        a_min, _ = self.get_parameter("amplitude_minimum", 0.1)
        a_max, _ = self.get_parameter("amplitude_maximum", 12)
        f_min, _ = self.get_parameter("frequency_minimum", 10)
        f_max, _ = self.get_parameter("frequency_maximum", 9000)
        n_max, _ = self.get_parameter("samples_maximum", 100)
        a = np.asarray(amplitudes, np.float64)
        f = np.abs(np.asarray(frequencies, np.float64))
        keep = (a >= float(a_min)) & (a <= float(a_max)) & (f >= float(f_min)) & (f <= float(f_max))
        a, f = a[keep], f[keep]
        order = np.argsort(-a, kind="stable")[:int(n_max)]
        return StreamEvent.OKAY, {"amplitudes": a[order], "frequencies": f[order]}


class PE_AudioResampler(PipelineElement):
    """Consolidate a spectrum into ``band_count`` bands (sum of amplitudes per band) over the
    positive half; optionally draws them on an LED matrix actor at ``led_topic`` with the
    reference's ``(led:fill ..)`` / ``(led:line ..)`` / ``(led:write)`` commands."""

    def __init__(self, context):
        context.set_protocol("audio_resample:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self.counter = 0

    def process_frame(self, stream, amplitudes, frequencies):
        bands, _ = self.get_parameter("band_count", 8)
        f_max, _ = self.get_parameter("frequency_maximum", 8000)
        bands = int(bands)
        a = np.asarray(amplitudes, np.float64)
        f = np.asarray(frequencies, np.float64)
        half = len(a) // 2 if (len(f) and f.min() < 0) else len(a)
        a, f = a[:half], f[:half]
        edges = np.linspace(0.0, float(f_max), bands + 1)
        idx = np.searchsorted(edges, f, side="right") - 1
        ok = (idx >= 0) & (idx < bands)
        band_amplitudes = np.bincount(idx[ok], weights=a[ok], minlength=bands)
        band_frequencies = (edges[:-1] + edges[1:]) / 2
        led_topic, _ = self.get_parameter("led_topic", None)
        self.counter += 1
        if led_topic:
            from ...runtime.process import aiko
            aiko.message.publish(led_topic, "(led:fill 0 0 0)")
            for x, amplitude in enumerate(band_amplitudes):
                aiko.message.publish(led_topic, f"(led:line 255 0 0 {x} 0 {x} {amplitude:.0f})")
            aiko.message.publish(led_topic, "(led:write)")
        return StreamEvent.OKAY, {"amplitudes": band_amplitudes, "frequencies": band_frequencies}


def render_xy(xs, ys, width=640, height=480, x_max=None, y_max=None, color=(0, 255, 0)):
    """Scatter plot -> uint8 [height, width, 3] image (axes along the left / bottom edges)."""
    img = np.zeros((height, width, 3), np.uint8)
    img[height - 1, :] = 128
    img[:, 0] = 128
    xs = np.abs(np.asarray(xs, np.float64))
    ys = np.asarray(ys, np.float64)
    if xs.size:
        x_max = float(x_max or xs.max() or 1.0)
        y_max = float(y_max or ys.max() or 1.0)
        px = np.clip((xs / x_max * (width - 1)).astype(int), 0, width - 1)
        py = np.clip(((1.0 - ys / y_max) * (height - 1)).astype(int), 0, height - 1)
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                img[np.clip(py + dy, 0, height - 1), np.clip(px + dx, 0, width - 1)] = color
    return img


class PE_GraphXY(PipelineElement):
    """Spectrum scatter graph as an ``image`` (render with VideoShow / ImageWriteFile)."""

    def __init__(self, context):
        context.set_protocol("graph_xy:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, amplitudes, frequencies):
        w, _ = self.get_parameter("width", 640)
        h, _ = self.get_parameter("height", 480)
        f_max, _ = self.get_parameter("frequency_maximum", 9000)
        a_max, _ = self.get_parameter("amplitude_maximum", 12)
        image = render_xy(frequencies, amplitudes, int(w), int(h), float(f_max), float(a_max))
        return StreamEvent.OKAY, {"amplitudes": amplitudes, "frequencies": frequencies, "image": image}


# ---- remote send / receive over binary MQTT topics (reference dead PE_RemoteSend*/Receive*) ----

def encode_array(array) -> bytes:
    """``zlib(np.save(array))`` — the reference's binary payload, without pickling."""
    buf = BytesIO()
    np.save(buf, np.asarray(array), allow_pickle=False)
    return zlib.compress(buf.getvalue(), 1)


def decode_array(payload: bytes) -> np.ndarray:
    return np.load(BytesIO(zlib.decompress(payload)), allow_pickle=False)


def _audio_topic(name: str) -> str:
    from ...utils.configuration import get_namespace
    return f"{get_namespace()}/audio/{name[-1]}"


class PE_RemoteSend0(PipelineElement):
    """Publish each frame's ``audio`` on ``{namespace}/audio/{last char of element name}``."""
    PARAMETER = "audio"

    def __init__(self, context):
        context.set_protocol("remote_send:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        topic, found = self.get_parameter("topic_audio", None)
        self.share["topic_audio"] = topic if found and topic else _audio_topic(self.name)

    def process_frame(self, stream, **inputs):
        from ...runtime.process import aiko
        value = inputs.get(self.PARAMETER)
        if value is None:
            value = next(iter(inputs.values()), "")
        aiko.message.publish(self.share["topic_audio"], encode_array(value))
        return StreamEvent.OKAY, {}


class PE_RemoteSend1(PE_RemoteSend0):
    pass


class PE_RemoteSend2(PE_RemoteSend0):
    PARAMETER = "text"


class PE_RemoteReceive0(PipelineElement):
    """Subscribe to the binary audio topic; every payload becomes a new frame on stream
    ``stream_id`` (parameter, default "0") carrying ``audio`` (``text`` for Receive2)."""
    PARAMETER = "audio"

    def __init__(self, context):
        context.set_protocol("remote_receive:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        topic, found = self.get_parameter("topic_audio", None)
        self.share["topic_audio"] = topic if found and topic else _audio_topic(self.name)
        self.share["frame_id"] = 0
        self.add_message_handler(self._receive, self.share["topic_audio"], binary=True)

    def _receive(self, _aiko, topic, payload_in):
        try:
            value = decode_array(payload_in)
        except (zlib.error, ValueError, OSError) as exc:
            self.logger.warning(f"{self.my_id()}: bad payload on {topic}: {exc}")
            return
        if self.PARAMETER == "text":
            value = str(value)
        frame_id = int(self.share["frame_id"])
        self.ec_producer.update("frame_id", frame_id + 1)
        stream_id, _ = self.get_parameter("stream_id", "0")
        self.pipeline.create_frame({"stream_id": str(stream_id), "frame_id": frame_id},
                                   {self.PARAMETER: value})

    def process_frame(self, stream, audio):
        return StreamEvent.OKAY, {"audio": audio}


class PE_RemoteReceive1(PE_RemoteReceive0):
    pass


class PE_RemoteReceive2(PE_RemoteReceive0):
    PARAMETER = "text"

    def process_frame(self, stream, text):
        text = str(text)
        return StreamEvent.OKAY, {"text": text or None}


# ---- device audio (sounddevice / pyaudio are optional) ---------------------------------------

def _import_audio_backend(name):
    try:
        return __import__(name)
    except ImportError as exc:
        raise RuntimeError(f"{name} is not installed: device audio elements need it "
                           f"(use AudioReadFile / AudioSynthetic / PE_RemoteReceive0 instead)") from exc


class _Microphone(PipelineElement):
    """Captures ``chunk_duration`` s chunks on a thread and emits them as frames of stream 0."""
    BACKEND = "sounddevice"

    def __init__(self, context):
        context.set_protocol("microphone:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self._backend = _import_audio_backend(self.BACKEND)
        self.share["frame_id"] = -1
        self.share["mute"] = 0
        self._time_mute = 0.0
        self.terminate = False

    def start_stream(self, stream, stream_id):
        self.terminate = False
        threading.Thread(target=self._audio_run, args=(stream,), daemon=True).start()
        return StreamEvent.OKAY, {}

    def _emit(self, stream, audio):
        if self._time_mute and time.time() < self._time_mute:
            return
        if self._time_mute:
            self._time_mute = 0.0
            self.ec_producer.update("mute", 0)
        frame_id = int(self.share["frame_id"]) + 1
        self.ec_producer.update("frame_id", frame_id)
        self.create_frame(stream, {"audio": audio}, frame_id=frame_id)

    def _audio_run(self, stream):
        rate, _ = self.get_parameter("sample_rate", 16000)
        dur, _ = self.get_parameter("chunk_duration", 5.0)
        channels, _ = self.get_parameter("audio_channels", 1)
        n = int(int(rate) * float(dur))
        sd = self._backend
        with sd.InputStream(channels=int(channels), samplerate=int(rate), dtype="float32") as s:
            while not self.terminate:
                data, _ = s.read(n)
                self._emit(stream, np.asarray(data, np.float32).mean(axis=1))

    def mute(self, duration):
        duration = float(duration)
        self._time_mute = time.time() + duration if duration else 0.0
        self.ec_producer.update("mute", duration)

    def process_frame(self, stream, audio):
        return StreamEvent.OKAY, {"audio": audio}

    def stop_stream(self, stream, stream_id):
        self.terminate = True
        return StreamEvent.OKAY, {}


class PE_MicrophoneSD(_Microphone):
    BACKEND = "sounddevice"


class PE_MicrophonePA(_Microphone):
    BACKEND = "pyaudio"

    def _audio_run(self, stream):
        rate, _ = self.get_parameter("sample_rate", 16000)
        dur, _ = self.get_parameter("chunk_duration", 2.0)
        channels, _ = self.get_parameter("audio_channels", 1)
        n = int(int(rate) * float(dur))
        pa = self._backend.PyAudio()
        s = pa.open(channels=int(channels), format=self._backend.paInt16, frames_per_buffer=n,
                    input=True, rate=int(rate))
        try:
            while not self.terminate:
                raw = np.frombuffer(s.read(n), dtype=np.int16).astype(np.float32) / 32768.0
                self._emit(stream, raw.reshape(-1, int(channels)).mean(axis=1))
        finally:
            s.close()
            pa.terminate()


class PE_Speaker(PipelineElement):
    """Play each ``audio`` frame (float32 at ``sample_rate``) through sounddevice."""

    def __init__(self, context):
        context.set_protocol("speaker:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self._sd = _import_audio_backend("sounddevice")

    def process_frame(self, stream, audio):
        rate, _ = self.get_parameter("sample_rate", 16000)
        self._sd.play(np.asarray(audio, np.float32), int(rate), blocking=True)
        return StreamEvent.OKAY, {}
