"""Native (HIP / gfx950) operator library of aiko_services_amd.

The kernels in ``aiko_services_amd/csrc`` are linked into ``aiko_services_amd/_C.so`` and
registered as ``torch.ops.aiko.*``.  :func:`load_native` loads that library once; on a GPU
box every op *requires* it — there is no silent eager fallback (``require_native``).  Torch
reference implementations used by the tests live in :mod:`aiko_services_amd.ops.reference`.
"""
from __future__ import annotations

import os
import threading
from pathlib import Path

import torch

_LIB = Path(__file__).resolve().parent.parent / "_C.so"
_lock = threading.Lock()
_loaded = False
_error: str | None = None


def native_library_path() -> Path:
    return _LIB


def load_native(build_if_missing: bool = False) -> bool:
    """Load ``_C.so`` (optionally building it first).  Returns True when loaded."""
    global _loaded, _error
    with _lock:
        if _loaded:
            return True
        if not _LIB.exists() and build_if_missing:
            from ..csrc.build import build
            build(verbose=False)
        if not _LIB.exists():
            _error = f"native library not built: {_LIB} (run python -m aiko_services_amd.csrc.build)"
            return False
        try:
            torch.ops.load_library(str(_LIB))
        except Exception as exc:  # pragma: no cover - depends on the box
            _error = f"failed to load {_LIB}: {exc}"
            return False
        _loaded = True
        return True


def native_available() -> bool:
    return load_native(build_if_missing=False)


def require_native() -> None:
    """Raise loudly if the HIP library is not loaded (never fall back to eager torch)."""
    if not load_native(build_if_missing=os.environ.get("AIKO_BUILD_ON_DEMAND", "1") == "1"):
        raise RuntimeError(f"aiko_services_amd native ops unavailable: {_error}")


from .conv import (ConvSpec, conv2d, linear, make_conv_spec, make_linear_spec,  # noqa: E402
                   make_stem_spec, stem_geometry)
from .vision import avgpool, maxpool2d, preprocess_frames, softmax_topk  # noqa: E402

__all__ = [
    "ConvSpec", "avgpool", "conv2d", "linear", "load_native", "make_conv_spec",
    "make_linear_spec", "make_stem_spec", "maxpool2d", "native_available",
    "native_library_path", "preprocess_frames", "require_native", "softmax_topk",
    "stem_geometry",
]
