"""Streams, frames and stream events (reference ``main/stream.py:30-98``).

A :class:`Stream` holds per-stream state (id, current frame id, graph path, parameters, the
response route) and its in-flight :class:`Frame` s; a frame's ``swag`` is the blackboard of
named values produced by elements — on the GPU path those values are device tensors (or
frame-pool slot handles) passed by reference, never serialised.
"""
from __future__ import annotations

import queue
from dataclasses import dataclass, field
from typing import Any, Dict

__all__ = ["DEFAULT_STREAM_ID", "FIRST_FRAME_ID", "Frame", "Stream", "StreamEvent",
           "StreamEventName", "StreamState", "StreamStateName"]

DEFAULT_STREAM_ID = "*"
FIRST_FRAME_ID = 0


class StreamEvent:
    ERROR = -2        # -> StreamState.ERROR
    STOP = -1         # -> StreamState.STOP
    OKAY = 0          # keep on running
    DROP_FRAME = 1    # stop processing this frame, keep running
    USER = 1024


StreamEventName = {
    StreamEvent.DROP_FRAME: "DropFrame",
    StreamEvent.ERROR: "Error",
    StreamEvent.OKAY: "Okay",
    StreamEvent.STOP: "Stop",
    StreamEvent.USER: "User",
}


class StreamState:
    ERROR = -2        # generate no new frames, ignore queued frames
    STOP = -1         # generate no new frames, process queued frames
    RUN = 0
    DROP_FRAME = 1
    USER = 1024


StreamStateName = {
    StreamState.DROP_FRAME: "DropFrame",
    StreamState.ERROR: "Error",
    StreamState.STOP: "Stop",
    StreamState.RUN: "Run",
    StreamState.USER: "User",
}


@dataclass
class Frame:
    metrics: Dict[str, Any] = field(default_factory=dict)
    paused_pe_name: str = None     # remote element awaited (continuation point)
    swag: Dict[str, Any] = field(default_factory=dict)
    hop_handles: list = field(default_factory=list)   # RCCL receive slots held by this frame
    hop_reply: int = None          # rank to send the response tensors to (remote hop)
    reply_to: str = None           # topic of the upstream stage that sent this frame
    on_complete: list = field(default_factory=list)   # callbacks when the frame completes
    lane: int = None               # frame lane (gpu_lanes > 1): a hop's response resumes on it


@dataclass
class Stream:
    stream_id: str = DEFAULT_STREAM_ID
    frame_id: int = FIRST_FRAME_ID
    graph_path: str = None
    frames: Dict[int, Frame] = field(default_factory=dict)
    parameters: Dict[str, Any] = field(default_factory=dict)
    queue_response: "queue.Queue" = None
    state: int = StreamState.RUN
    topic_response: str = None
    variables: Dict[str, Any] = field(default_factory=dict)

    def as_dict(self):
        return {"stream_id": self.stream_id, "frame_id": self.frame_id}

    def update(self, stream_dict):
        if not isinstance(stream_dict, dict):
            return False
        self.stream_id = str(stream_dict.get("stream_id", self.stream_id))
        self.frame_id = int(stream_dict.get("frame_id", self.frame_id))
        self.graph_path = stream_dict.get("graph_path", self.graph_path)
        self.parameters = stream_dict.get("parameters", self.parameters)
        self.state = int(stream_dict.get("state", StreamState.RUN))
        return True
