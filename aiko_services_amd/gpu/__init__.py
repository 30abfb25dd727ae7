"""GPU runtime: device binding, GPU-resident PipelineElements, HBM frame pools, results."""
from .device import device_info, gpu_available, parse_device, require_gpu, select_device  # noqa: F401
from .element import CapturedCall, DeviceResult, FramePool, GpuPipelineElement  # noqa: F401
