"""LLM example elements (reference ``examples/llm/elements_llm.py:191-220``): ``PE_LLM`` sends
the frame's ``text`` to an OpenAI-compatible chat endpoint (``url`` parameter; pass-through
without one).  LangChain / Ollama and Coqui TTS are not available offline and are not
reproduced; the element is shared with the speech example."""
from aiko_services_amd.examples.speech.speech_elements import PE_LLM

__all__ = ["PE_LLM"]
