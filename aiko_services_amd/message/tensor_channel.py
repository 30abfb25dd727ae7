"""TensorChannel: the data-plane counterpart of :class:`Message` (SURVEY C7 / P1 "D" rows).

Frame metadata keeps flowing as S-expressions on the MQTT control plane; tensor payloads move
over a TensorChannel:

* :class:`LoopbackTensorChannel` — same process: device tensors are handed over by reference
  (zero copy), ordered by a queue — used when producer and consumer stages share a GPU;
* :class:`RcclTensorChannel`     — another rank (one process per MI355X): RCCL point-to-point
  over xGMI through a :class:`~aiko_services_amd.parallel.pipeline_parallel.StageLink` (slot
  ring, signature negotiated on the first frame, grouped send/recv).

Both speak ``send(header, tensors)`` / ``recv() -> (header, tensors)`` where ``header`` is a
short list of ints (frame id, stream state, timestamp).
"""
from __future__ import annotations

import queue
from abc import ABC, abstractmethod

import torch

__all__ = ["TensorChannel", "LoopbackTensorChannel", "RcclTensorChannel"]


class TensorChannel(ABC):
    @abstractmethod
    def send(self, header, tensors: dict) -> None:
        pass

    @abstractmethod
    def recv(self, timeout: float | None = None):
        pass

    def close(self) -> None:
        pass


class LoopbackTensorChannel(TensorChannel):
    def __init__(self, maxsize: int = 0):
        self._q: queue.Queue = queue.Queue(maxsize)

    def send(self, header, tensors: dict) -> None:
        self._q.put((list(header), dict(tensors)))

    def recv(self, timeout: float | None = None):
        return self._q.get(timeout=timeout)


class RcclTensorChannel(TensorChannel):
    """One direction between this rank and ``peer``; ``role`` is "send" or "recv"."""

    def __init__(self, peer: int, role: str, device=None, depth: int = 2):
        from ..parallel.pipeline_parallel import StageLink
        if role not in ("send", "recv"):
            raise ValueError("role must be 'send' or 'recv'")
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.role = role
        self.link = StageLink(peer, device, depth)

    def send(self, header, tensors: dict) -> None:
        if self.role != "send":
            raise RuntimeError("send on a receive channel")
        self.link.send(header, tensors)

    def recv(self, timeout: float | None = None):
        if self.role != "recv":
            raise RuntimeError("recv on a send channel")
        slot = self.link.post_recv()
        hdr, bufs = self.link.wait(slot)
        return hdr.tolist(), dict(bufs)

    def close(self) -> None:
        self.link.drain()
