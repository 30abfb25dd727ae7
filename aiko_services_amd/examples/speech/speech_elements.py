"""Speech example elements under the reference's names (``examples/speech/speech_elements.py``:
PE_LLM :43, PE_AudioFraming :60, PE_AudioWriteFile :89, PE_SpeechFraming :150).

* ``PE_AudioFraming`` — LRU sliding window over the last ``window_chunks`` audio chunks
  (``audio``: ndarray or a WAV path, which is read and — like the reference — deleted when
  ``delete_input`` is true) -> concatenated ``audio``;
* ``PE_AudioWriteFile`` — ``audio`` -> ``y_audio_{frame_id:06}.wav`` (``path_template``);
* ``PE_SpeechFraming`` — text pass-through (segmenting hook);
* ``PE_LLM`` — text pass-through, or, with an ``url`` parameter, one chat-completion request to
  an OpenAI-compatible HTTP endpoint (``model``, ``timeout``) whose reply becomes ``text``.

The transcription model itself is the GPU ``WhisperEncoder`` element
(``elements/gpu/speech.py``); the reference's WhisperX / Coqui TTS need downloaded checkpoints
and are not reproduced.
"""
from __future__ import annotations

from collections import OrderedDict
import os

import numpy as np

from aiko_services_amd.elements.media.audio_io import read_wav, write_wav
from aiko_services_amd.pipeline.engine import PipelineElement
from aiko_services_amd.pipeline.stream import StreamEvent

__all__ = ["PE_AudioFraming", "PE_AudioWriteFile", "PE_SpeechFraming", "PE_LLM"]


class _Element(PipelineElement):
    PROTOCOL = "speech:0"

    def __init__(self, context):
        context.set_protocol(self.PROTOCOL)
        context.get_implementation("PipelineElement").__init__(self, context)


class PE_AudioFraming(_Element):
    PROTOCOL = "audio_framing:0"

    def start_stream(self, stream, stream_id):
        stream.variables["framing_lru"] = OrderedDict()
        return StreamEvent.OKAY, {}

    def process_frame(self, stream, audio):
        if isinstance(audio, (str, os.PathLike)):
            path = str(audio)
            audio, _rate = read_wav(path)
            if str(self.get_parameter("delete_input", False)[0]).lower() in ("true", "1"):
                os.remove(path)
        lru = stream.variables.setdefault("framing_lru", OrderedDict())
        lru[stream.frame_id] = np.asarray(audio, np.float32).reshape(-1)
        size = int(self.get_parameter("window_chunks", 1)[0])
        while len(lru) > size:
            lru.popitem(last=False)
        return StreamEvent.OKAY, {"audio": np.concatenate(list(lru.values()))}


class PE_AudioWriteFile(_Element):
    PROTOCOL = "audio_write_file:0"

    def process_frame(self, stream, audio):
        template = str(self.get_parameter("path_template", "y_audio_{frame_id:06}.wav")[0])
        path = template.format(frame_id=int(stream.frame_id))
        write_wav(path, np.asarray(audio, np.float32), int(self.get_parameter("sample_rate", 16000)[0]))
        return StreamEvent.OKAY, {"audio": path}


class PE_SpeechFraming(_Element):
    PROTOCOL = "speech_framing:0"

    def process_frame(self, stream, text):
        return StreamEvent.OKAY, {"text": text}


class PE_LLM(_Element):
    PROTOCOL = "llm:0"

    def process_frame(self, stream, text):
        url, found = self.get_parameter("url")
        if not found or not url:
            return StreamEvent.OKAY, {"text": text}
        import requests
        body = {"model": str(self.get_parameter("model", "default")[0]),
                "messages": [{"role": "user", "content": str(text)}]}
        try:
            r = requests.post(str(url), json=body, timeout=float(self.get_parameter("timeout", 30)[0]))
            r.raise_for_status()
            reply = r.json()["choices"][0]["message"]["content"]
        except Exception as exc:
            return StreamEvent.ERROR, {"diagnostic": f"PE_LLM request failed: {exc}"}
        return StreamEvent.OKAY, {"text": reply}
