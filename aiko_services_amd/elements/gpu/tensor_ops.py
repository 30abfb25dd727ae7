"""Small GPU tensor elements for data-plane tests and demos (branch concurrency on HIP streams).

* ``GpuTensorSource`` — fixed random bf16 matrix ``[size, size]`` per frame;
* ``GpuMatChain``     — ``repeat`` x (y = tanh(y @ W)); output name taken from the definition;
* ``GpuAdd``          — element-wise sum of its two declared inputs.

Give two branches of a diamond graph different ``hip_stream`` parameters and they overlap on
the GPU; the join waits on their events (``GpuPipelineElement.stream_enter``)."""
from __future__ import annotations

import torch

from ...gpu.element import GpuPipelineElement
from ...pipeline.stream import StreamEvent

__all__ = ["GpuTensorSource", "GpuMatChain", "GpuAdd"]


def _out_name(el, default):
    outs = el.definition.output or []
    return outs[0]["name"] if outs else default


class GpuTensorSource(GpuPipelineElement):
    def __init__(self, context):
        context.set_protocol("gpu_tensor_source:0")
        super().__init__(context)
        n = int(self.get_parameter("size", 1024)[0])
        g = torch.Generator(device=self.device).manual_seed(int(self.get_parameter("seed", 0)[0]))
        self.x = (torch.randn(n, n, device=self.device, generator=g) / n ** 0.5).to(torch.bfloat16)

    def process_frame(self, stream, **kwargs):
        return StreamEvent.OKAY, {_out_name(self, "x"): self.x}


class GpuMatChain(GpuPipelineElement):
    def __init__(self, context):
        context.set_protocol("gpu_mat_chain:0")
        super().__init__(context)
        self.repeat = int(self.get_parameter("repeat", 8)[0])
        self.w = None

    def process_frame(self, stream, x):
        if self.w is None or self.w.shape[0] != x.shape[1]:
            g = torch.Generator(device=self.device).manual_seed(int(self.get_parameter("seed", 1)[0]))
            n = x.shape[1]
            self.w = (torch.randn(n, n, device=self.device, generator=g) * (2.0 / n) ** 0.5).to(torch.bfloat16)
        y = x
        for _ in range(self.repeat):
            y = torch.tanh(y @ self.w)
        return StreamEvent.OKAY, {_out_name(self, "y"): y}


class GpuAdd(GpuPipelineElement):
    def __init__(self, context):
        context.set_protocol("gpu_add:0")
        super().__init__(context)

    def process_frame(self, stream, **inputs):
        a, b = list(inputs.values())[:2]
        return StreamEvent.OKAY, {_out_name(self, "z"): a + b}
