"""LLM example elements (reference ``examples/llm/elements_llm.py:68-220``).

``PE_LLM`` turns a transcribed utterance into a robot command S-expression with a chat model,
as the reference's LangChain chain does (``llm_chain``, ``:97-187``): a system prompt listing
the robot's actions, the user's text, temperature 0.  It adds the objects seen within the last
second, taken from the ``{namespace}/detections`` topic (``:197-209``), and passes
``<silence>`` through unchanged.

LangChain is not installed here, so the two backends it wraps are spoken to directly over HTTP:
* ``llm_type: ollama`` (the reference's default): ``POST {url}/api/chat``, with ``stream:
  false`` and ``options.temperature``; the reply is ``message.content``.  The default ``url`` is
  ``http://127.0.0.1:11434`` and the default model ``llama3.1:latest``.
* ``llm_type: openai``: ``POST {url}/chat/completions``.  The default ``url`` is
  ``https://api.openai.com/v1``, the bearer token comes from ``OPENAI_API_KEY``, and the reply is
  ``choices[0].message.content``.  This also reaches any OpenAI-compatible local server.
Parameters: ``llm_type``, ``url``, ``model``, ``temperature``, ``timeout``.  A failed request
ends the frame with an ERROR diagnostic.

``PE_COQUI_TTS`` is the reference's text pass-through stand-in for speech synthesis (``:68-74``).
"""
from __future__ import annotations

import os
import threading
import time

from ...pipeline.engine import PipelineElement
from ...pipeline.stream import StreamEvent
from ...utils.configuration import get_namespace

__all__ = ["PE_LLM", "PE_COQUI_TTS", "llm_chain", "llm_messages", "SYSTEM_PROMPT",
           "LLM_MODEL_NAME", "topic_detections"]

LLM_MODEL_NAME = "llama3.1:latest"
LLM_TEMPERATURE = 0.0
DETECTIONS_MAX_AGE_S = 1.0
_DEFAULT_URL = {"ollama": "http://127.0.0.1:11434", "openai": "https://api.openai.com/v1"}

# The robot's command vocabulary (reference SYSTEM_PROMPT, :137-178): the model must answer with
# one S-expression — an action, a query, a short response, or an error.
_ACTIONS = ["select all", "select bruce", "select oscar", "select none", "arm lower", "arm raise",
            "backwards", "crawl", "forwards", "hand close", "hand open", "pee", "pitch down",
            "pitch up", "reset", "sit", "sniff", "stop", "stretch", "turn left", "turn right", "wag"]
SYSTEM_PROMPT = "\n".join(
    ["Answer only with one valid S-expression, without explanation or examples.",
     "Commands map to one of:"]
    + [f"- (action {a})" for a in _ACTIONS]
    + ["Questions about the weather map to:",
       "- (get_temperature location)  ;; e.g. location = Melbourne",
       "Any other conversation maps to:",
       "- (response message)  ;; at most 12 words",
       "When unsure, reply:",
       "- (error diagnostic_message)",
       'Call the robot a "robot dog", never "xgomini2".',
       "Facts about yourself, for responses: name Oscar; type xgomini2 robot dog; goal: being "
       "happy; interests: fetching balls; best friend: octopus"])


def topic_detections() -> str:
    return f"{get_namespace()}/detections"


def llm_messages(text: str, detections="") -> list:
    """System + user chat messages; ``detections`` (objects currently seen) extend the system
    prompt."""
    seen = " ".join(detections) if isinstance(detections, (list, tuple)) else str(detections or "")
    return [{"role": "system", "content": SYSTEM_PROMPT + f"\n- currently seen: {seen}"},
            {"role": "user", "content": str(text)}]


def llm_chain(llm_type: str, text: str, detections="", url: str | None = None,
              model: str = LLM_MODEL_NAME, temperature: float = LLM_TEMPERATURE,
              timeout: float = 60.0) -> str:
    """One chat request to an Ollama or OpenAI(-compatible) server; returns the reply text."""
    import requests
    messages = llm_messages(text, detections)
    if llm_type == "ollama":
        base = (url or _DEFAULT_URL["ollama"]).rstrip("/")
        r = requests.post(f"{base}/api/chat", timeout=timeout,
                          json={"model": model, "messages": messages, "stream": False,
                                "options": {"temperature": float(temperature)}})
        r.raise_for_status()
        return str(r.json()["message"]["content"])
    if llm_type == "openai":
        base = (url or _DEFAULT_URL["openai"]).rstrip("/")
        headers = {}
        if os.environ.get("OPENAI_API_KEY"):
            headers["Authorization"] = f"Bearer {os.environ['OPENAI_API_KEY']}"
        endpoint = base if base.endswith("/chat/completions") else f"{base}/chat/completions"
        r = requests.post(endpoint, timeout=timeout, headers=headers,
                          json={"model": model, "messages": messages, "temperature": float(temperature)})
        r.raise_for_status()
        return str(r.json()["choices"][0]["message"]["content"])
    raise ValueError(f"Unknown llm_type: {llm_type} (ollama | openai)")


class PE_COQUI_TTS(PipelineElement):
    def __init__(self, context):
        context.set_protocol("text_to_speech:0")
        context.get_implementation("PipelineElement").__init__(self, context)

    def process_frame(self, stream, text):
        return StreamEvent.OKAY, {"text": text}


class PE_LLM(PipelineElement):
    def __init__(self, context):
        context.set_protocol("llm:0")
        context.get_implementation("PipelineElement").__init__(self, context)
        self._lock = threading.Lock()
        self.detections = None                     # (time received, [object names])
        try:
            self.add_message_handler(self.detection_handler, topic_detections())
        except Exception as exc:                    # no message transport (bare unit use)
            self.logger.debug(f"PE_LLM: no detections subscription: {exc}")

    def detection_handler(self, _aiko, topic, payload_in):
        words = str(payload_in).split()
        with self._lock:
            self.detections = (time.time(), words[1:])

    def recent_detections(self):
        with self._lock:
            if not self.detections:
                return ""
            when, names = self.detections
        return names if time.time() <= when + DETECTIONS_MAX_AGE_S else ""

    def process_frame(self, stream, text):
        if text == "<silence>":
            return StreamEvent.OKAY, {"text": text}
        p = lambda name, default: self.get_parameter(name, default)[0]   # noqa: E731
        self.logger.info(f"Input: {text}")
        try:
            reply = llm_chain(str(p("llm_type", "ollama")), text, self.recent_detections(),
                              url=p("url", None), model=str(p("model", LLM_MODEL_NAME)),
                              temperature=float(p("temperature", LLM_TEMPERATURE)),
                              timeout=float(p("timeout", 60)))
        except Exception as exc:
            return StreamEvent.ERROR, {"diagnostic": f"PE_LLM request failed: {exc}"}
        return StreamEvent.OKAY, {"text": reply}
