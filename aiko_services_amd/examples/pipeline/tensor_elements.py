"""Deterministic tensor PipelineElements for multi-process / multi-GPU pipeline tests.

They run on the element's ``device`` (``"cpu"`` for the gloo tests, a GPU otherwise) and are
bit-reproducible, so a pipeline split over processes (``parallel/placement.py``, remote hops
over RCCL / gloo) must produce exactly the outputs of the single-process run.

* ``TensorFrames`` — frame generator (``frames`` per stream): ``x`` float32 [batch, width],
  a function of the frame id, plus ``t_submit`` (``gpu_sleep``: GPU cycles spent before ``x``
  is written — a slow producer for stream-ordering tests);
* ``TensorAffine`` — ``x * scale + shift`` (float32, element-wise);
* ``TensorStats``  — per-row sum and max as a :class:`DeviceResult` (``stats``).
"""
from __future__ import annotations

import time

import torch

from ...gpu.element import DeviceResult, GpuPipelineElement
from ...pipeline.stream import StreamEvent

__all__ = ["TensorFrames", "TensorAffine", "TensorStats"]


class TensorFrames(GpuPipelineElement):
    lane_safe = True          # no device state kept across frames

    def __init__(self, context):
        context.set_protocol("tensor_frames:0")
        super().__init__(context)

    def start_stream(self, stream, stream_id):
        limit, found = self.get_parameter("frames")
        if found and limit:
            stream.variables["tensor_frames_left"] = int(limit)
            rate, _ = self.get_parameter("rate")          # frames per second (None: as fast as admitted)
            self.create_frames(stream, self.frame_generator, rate=float(rate) if rate else None)
        return StreamEvent.OKAY, None

    def frame_generator(self, stream, frame_id):
        left = stream.variables.get("tensor_frames_left", 0)
        if left <= 0:
            return StreamEvent.STOP, {"diagnostic": "All frames generated"}
        stream.variables["tensor_frames_left"] = left - 1
        return StreamEvent.OKAY, {"t_submit": time.perf_counter()}

    def process_frame(self, stream, **kwargs):
        _, frame_id = self.get_stream()
        B = int(self.get_parameter("batch", 4)[0])
        W = int(self.get_parameter("width", 256)[0])
        sleep = int(self.get_parameter("gpu_sleep", 0)[0] or 0)
        if sleep and self.device.type == "cuda":
            # a slow producer (GPU cycles before x is written): stream-ordering tests
            torch.cuda._sleep(sleep)
        x = torch.arange(B * W, dtype=torch.float32, device=self.device).reshape(B, W)
        x = torch.sin(x * 0.01 + float(frame_id))
        return StreamEvent.OKAY, {"x": x, "t_submit": kwargs.get("t_submit", time.perf_counter())}


class TensorAffine(GpuPipelineElement):
    lane_safe = True          # no device state kept across frames

    def __init__(self, context):
        context.set_protocol("tensor_affine:0")
        super().__init__(context)

    def process_frame(self, stream, x):
        scale = float(self.get_parameter("scale", 2.0)[0])
        shift = float(self.get_parameter("shift", 0.5)[0])
        return StreamEvent.OKAY, {"x": x * scale + shift}


class TensorStats(GpuPipelineElement):
    lane_safe = True          # no device state kept across frames

    def __init__(self, context):
        context.set_protocol("tensor_stats:0")
        super().__init__(context)

    def process_frame(self, stream, x, t_submit=None):
        s, m = x.sum(dim=1), x.amax(dim=1)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        return StreamEvent.OKAY, {"stats": DeviceResult({"sum": s, "max": m}, ev,
                                                        t_submit=t_submit if isinstance(t_submit, float) else None)}
