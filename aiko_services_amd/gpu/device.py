"""GPU device binding for GPU-resident actors: one process per MI355X.

``select_device()`` resolves the device of this process (``AIKO_GPU_DEVICE`` >
``AIKO_GPU_DEVICE_MAP[LOCAL_RANK]`` > ``LOCAL_RANK`` > 0), binds it, applies
``AIKO_GPU_MEMORY_FRACTION`` and returns a ``torch.device``.  ``require_gpu()`` fails loudly
when no HIP device is visible — GPU elements never silently fall back to the CPU.
"""
from __future__ import annotations

import os

import torch

from ..utils.configuration import get_gpu_configuration

__all__ = ["select_device", "require_gpu", "gpu_available", "parse_device", "device_info"]


def gpu_available() -> bool:
    return torch.cuda.is_available()


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("aiko_services_amd: this element needs an MI355X (HIP) device, none visible")


def parse_device(spec) -> torch.device:
    """``"gpu:3"`` / ``"cuda:3"`` / ``3`` / ``None`` -> torch.device (None = this process's GPU)."""
    if spec is None or spec == "" or spec == "gpu":
        return select_device()
    if isinstance(spec, int) or (isinstance(spec, str) and spec.isdigit()):
        return torch.device("cuda", int(spec))
    s = str(spec)
    if s.startswith("gpu:"):
        return torch.device("cuda", int(s.split(":", 1)[1]))
    return torch.device(s)


_selected = None


def select_device() -> torch.device:
    global _selected
    if _selected is None:
        require_gpu()
        cfg = get_gpu_configuration()
        idx = cfg.device_for_local_rank(int(os.environ.get("LOCAL_RANK", "0")))
        idx = idx % max(1, torch.cuda.device_count())
        torch.cuda.set_device(idx)
        if cfg.memory_fraction < 1.0:
            torch.cuda.set_per_process_memory_fraction(cfg.memory_fraction, idx)
        _selected = torch.device("cuda", idx)
    return _selected


def device_info(device=None) -> dict:
    if not torch.cuda.is_available():
        return {"available": False}
    device = device or torch.device("cuda", torch.cuda.current_device())
    p = torch.cuda.get_device_properties(device)
    free, total = torch.cuda.mem_get_info(device)
    return {"available": True, "name": p.name, "arch": getattr(p, "gcnArchName", "?"),
            "cus": p.multi_processor_count, "hbm_total_gb": total / 2**30, "hbm_free_gb": free / 2**30}
