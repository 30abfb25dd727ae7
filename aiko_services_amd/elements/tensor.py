"""Device-agnostic tensor PipelineElements: building blocks for data-plane tests and examples
(pipeline/data parallel runners on CPU with gloo, or on MI355X with RCCL).

* ``TensorSource``  — emits ``x`` = frame_id + arange(size) (float32, shape [batch, size]);
* ``TensorAffine``  — ``x * scale + offset``;
* ``TensorReduce``  — ``sum`` over the last dim -> ``y`` [batch];
* ``TensorDrop``    — DROP_FRAME every ``every``-th frame (stream-state propagation tests).
"""
from __future__ import annotations

import torch

from ..pipeline.engine import PipelineElement
from ..pipeline.stream import StreamEvent

__all__ = ["TensorSource", "TensorAffine", "TensorReduce", "TensorDrop", "FrameStats", "TensorEcho"]


class _TensorElement(PipelineElement):
    PROTOCOL = "tensor:0"

    def __init__(self, context):
        context.set_protocol(self.PROTOCOL)
        context.get_implementation("PipelineElement").__init__(self, context)
        dev, _ = self.get_parameter("device", default=None)
        deploy = getattr(self.definition, "deploy", None)
        dev = dev or getattr(deploy, "device", None)
        if dev is None:
            dev = f"cuda:{torch.cuda.current_device()}" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(str(dev).replace("gpu:", "cuda:"))

    def start_stream(self, stream, stream_id):
        return StreamEvent.OKAY, None


class TensorSource(_TensorElement):
    PROTOCOL = "tensor_source:0"

    def process_frame(self, stream, **kwargs):
        batch = int(self.get_parameter("batch", 2)[0])
        size = int(self.get_parameter("size", 8)[0])
        base = torch.arange(size, dtype=torch.float32, device=self.device)
        x = (base + float(stream.frame_id)).expand(batch, size).contiguous()
        return StreamEvent.OKAY, {"x": x}


class TensorAffine(_TensorElement):
    PROTOCOL = "tensor_affine:0"

    def process_frame(self, stream, x):
        scale = float(self.get_parameter("scale", 1.0)[0])
        offset = float(self.get_parameter("offset", 0.0)[0])
        return StreamEvent.OKAY, {"x": x * scale + offset}


class TensorReduce(_TensorElement):
    PROTOCOL = "tensor_reduce:0"

    def process_frame(self, stream, x):
        return StreamEvent.OKAY, {"y": x.sum(dim=-1)}


class TensorDrop(_TensorElement):
    PROTOCOL = "tensor_drop:0"

    def process_frame(self, stream, x):
        every = int(self.get_parameter("every", 0)[0])
        if every and stream.frame_id % every == every - 1:
            return StreamEvent.DROP_FRAME, {"x": x}
        return StreamEvent.OKAY, {"x": x}


class FrameStats(_TensorElement):
    """Stand-in detector for data-plane tests: uint8 frames [B, H, W, 3] -> fixed-size
    "detections" [B, 1, 6] (per-frame channel means, frame mean, 0) + counts [B] (= 1)."""
    PROTOCOL = "frame_stats:0"

    def process_frame(self, stream, images):
        f = images.float()
        ch = f.mean(dim=(1, 2))                                   # [B, 3]
        det = torch.zeros(images.shape[0], 1, 6, device=images.device)
        det[:, 0, :3] = ch
        det[:, 0, 3] = f.mean(dim=(1, 2, 3))
        counts = torch.ones(images.shape[0], dtype=torch.int32, device=images.device)
        return StreamEvent.OKAY, {"detections": det, "counts": counts}


class TensorEcho(PipelineElement):
    """Remote-hop test element: returns its array inputs unchanged plus exact derived values
    (``x2`` = 2 x, ``u_sum``), on whatever device / container they arrived in (torch tensor or
    numpy array) — the far end of the binary tensor-payload path (``message/tensor_payload.py``)."""
    PROTOCOL = "tensor_echo:0"

    def __init__(self, context):
        context.set_protocol(self.PROTOCOL)
        context.get_implementation("PipelineElement").__init__(self, context)

    def start_stream(self, stream, stream_id):
        return StreamEvent.OKAY, None

    def process_frame(self, stream, x, u):
        device = str(x.device) if isinstance(x, torch.Tensor) else "numpy"
        return StreamEvent.OKAY, {"x": x, "u": u, "x2": x * 2, "u_sum": int(u.astype("int64").sum()),
                                  "device_in": device}
