"""Torch-free half of the hop plane (``parallel/hop.py``): the process-wide plane handle, the
failure exceptions and the message-token predicates.  The pipeline engine imports THIS module,
so control-plane processes (registrar, CPU-only reference pipelines, brokers) never load torch;
``parallel.hop`` (torch + torch.distributed) is imported only where a plane is created."""
from __future__ import annotations

__all__ = ["StageFailure", "NoCredit", "plane", "set_plane", "is_token", "needs_decode", "TOKEN",
           "FLOAT_TOKEN", "RESULT_KEY"]

TOKEN = "T@"
FLOAT_TOKEN = "F@"
RESULT_KEY = "_device_result"

_plane = None


class StageFailure(RuntimeError):
    """A peer rank of the hop plane is gone (registrar removal, last will or transport error)."""

    def __init__(self, peer: int, cause=None):
        super().__init__(f"hop: stage rank {peer} failed" + (f": {cause}" if cause else ""))
        self.peer = peer


class NoCredit(RuntimeError):
    """Every staging slot toward the peer holds an unacknowledged frame."""


def plane():
    """The process's :class:`~aiko_services_amd.parallel.hop.HopPlane`, or None."""
    return _plane


def set_plane(p) -> None:
    global _plane
    _plane = p


def is_token(v) -> bool:
    return isinstance(v, str) and (v.startswith(TOKEN) or v.startswith(FLOAT_TOKEN))


def needs_decode(stream_dict, values) -> bool:
    """Whether a ``process_frame`` / ``process_frame_response`` message went through
    :meth:`HopPlane.encode`: the stream dict names a hop rank (forward hops), or a value is a
    tensor / float token or an encoded DeviceResult (responses).  Plain nested-dict swag values
    of reference pipelines never enter the token scanner."""
    if isinstance(stream_dict, dict) and stream_dict.get("hop_rank") is not None:
        return True
    if not isinstance(values, dict):
        return False
    for v in values.values():
        if is_token(v) or (isinstance(v, dict) and RESULT_KEY in v):
            return True
    return False
