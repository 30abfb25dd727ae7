"""Frame lanes: successive frames of a GPU pipeline on alternating HIP streams.

A pipeline with ``gpu_lanes: N`` (definition / stream parameter, default ``AIKO_GPU_LANES``)
runs frame k entirely on lane ``k % N``: every element's launches (or hipGraph replay) go to
that lane's HIP stream, and lane-aware elements keep one workspace / captured graph / output
buffer set per lane.  Consecutive frames are then independent chains on different streams,
so the GPU overlaps frame k's tail with frame k+1's head — a memory-bound early stage of one
frame runs next to a compute-bound late stage of the other, and the inter-kernel gaps and
last-wave tails of a single in-order chain get filled (ResNet-50 B=256 on one MI355X:
54.5k -> 62k frames/s with 2 lanes, ``scripts/r50_lanes.py``).  This is the GPU form of the
reference's concurrent frames per stream.

Results stay correct because every buffer a lane writes is private to it; buffers shared
across frames (read-only frame pools, pinned host result rings) are safe as long as fewer
frames are in flight than ring slots.  An element declares ``lane_safe = True`` once it keys
its mutable device state by :func:`current_lane`; the engine refuses ``gpu_lanes > 1`` for a
pipeline containing a GPU element that has not.
"""
from __future__ import annotations

import threading

__all__ = ["current_lane", "in_lane", "lane_scope", "lane_stream"]

_tls = threading.local()
_STREAMS: dict = {}


def current_lane() -> int:
    """Lane index of the frame being processed on this thread (0 outside lanes)."""
    return getattr(_tls, "lane", 0)


def in_lane() -> bool:
    """Whether this thread is inside a :class:`lane_scope` (a nested pipeline — e.g. rank 0's
    local share of a replicated stage — then keeps the enclosing frame's lane)."""
    return getattr(_tls, "depth", 0) > 0


def lane_stream(device, lane: int):
    import torch
    key = (str(device), lane)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(device=device)
    return st


class lane_scope:
    """Run the enclosed launches on lane ``lane``'s stream; the lane stream first waits for
    the work already queued on the current stream (frame inputs), and on exit the current
    stream is NOT made to wait — results carry their own events (``DeviceResult``)."""

    def __init__(self, lane: int, device):
        self.lane = lane
        self.device = device
        self._ctx = None
        self._prev = 0

    def __enter__(self):
        import torch
        st = lane_stream(self.device, self.lane)
        st.wait_stream(torch.cuda.current_stream(self.device))
        self._ctx = torch.cuda.stream(st)
        self._ctx.__enter__()
        self._prev = current_lane()
        _tls.lane = self.lane
        _tls.depth = getattr(_tls, "depth", 0) + 1
        return self

    def __exit__(self, *exc):
        _tls.lane = self._prev
        _tls.depth -= 1
        self._ctx.__exit__(*exc)
        return False
