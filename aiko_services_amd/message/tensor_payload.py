"""Binary control-plane messages that carry tensors: the MQTT path for array payloads that do not
ride an RCCL hop plan.

The reference ships arrays between processes as binary MQTT payloads, ``zlib(np.save(array))``
(``/root/reference/src/aiko_services/examples/xgo_robot/xgo_robot.py:320-324``), and its remote
pipeline hop publishes the element inputs with ``generate()``
(``/root/reference/src/aiko_services/main/pipeline.py:1080-1090``).  Here every remote method call
and every ``/out`` publication goes through :func:`encode_message`:

* no array anywhere in the parameters  -> the plain S-expression text (unchanged wire format);
* any ``torch.Tensor`` / ``numpy.ndarray`` / :class:`~aiko_services_amd.gpu.element.DeviceResult`
  -> ONE binary payload::

      MAGIC | u32 header length | header (JSON) | pad to 64 | blob 0 | pad | blob 1 ...

  The header holds the S-expression with every array replaced by ``0:`` (None) and, per array,
  its path inside the parsed message, kind (torch / numpy), dtype, shape, source device, and
  the blob's offset / length / codec (``raw``, or ``zlib`` with ``AIKO_TENSOR_ZLIB=1`` as the
  reference does).  Blobs are the array's bytes in C order (bf16 and other dtypes numpy lacks
  travel as torch bytes); nothing is pickled, so a decoder executes nothing from the wire.

:func:`~aiko_services_amd.utils.sexpr.parse` recognises the magic and returns the decoded
``(command, parameters)`` with the arrays in place: a device tensor comes back on the
receiver's current GPU (host-staged; on-node GPU peers in an RCCL plan use ``parallel/hop.py``
instead), a CPU tensor / ndarray on the host, bit-exact.  ``generate()`` itself refuses arrays
(``TypeError``): an array is never rendered with ``str()``.
"""
from __future__ import annotations

import json
import math
import os
import struct
import sys
import zlib

import numpy as np

from ..utils.sexpr import generate

__all__ = ["MAGIC", "encode_message", "decode_message", "is_tensor_payload", "has_arrays",
           "is_array"]

MAGIC = b"\x00AIKO-TP1\n"
_ALIGN = 64
_CODEC = "zlib" if os.environ.get("AIKO_TENSOR_ZLIB", "0") not in ("0", "", "false") else "raw"


def _torch():
    return sys.modules.get("torch")


def _is_torch_tensor(x) -> bool:
    t = _torch()
    return t is not None and isinstance(x, t.Tensor)


def _is_device_result(x) -> bool:
    return getattr(type(x), "__aiko_device_result__", False)


def is_array(x) -> bool:
    return isinstance(x, np.ndarray) or _is_torch_tensor(x) or _is_device_result(x)


def has_arrays(obj) -> bool:
    if is_array(obj):
        return True
    if isinstance(obj, dict):
        return any(has_arrays(v) for v in obj.values())
    if isinstance(obj, (list, tuple)):
        return any(has_arrays(v) for v in obj)
    return False


def is_tensor_payload(payload) -> bool:
    return isinstance(payload, (bytes, bytearray, memoryview)) and bytes(payload[:len(MAGIC)]) == MAGIC


def _host_bytes(x):
    """(kind, dtype name, shape, device, memoryview of the C-order bytes) of one array."""
    if isinstance(x, np.ndarray):
        if x.dtype.hasobject:
            raise TypeError("object arrays cannot be sent (nothing is pickled)")
        a = np.ascontiguousarray(x)
        return "numpy", a.dtype.str, list(a.shape), "cpu", memoryview(a.reshape(-1).view(np.uint8))
    t = x.detach()
    device = str(t.device)
    if t.device.type != "cpu":
        t = t.to("cpu")                               # staged through host memory (synchronous)
    t = t.contiguous()
    raw = t.reshape(-1).view(_torch().uint8).numpy()
    return "torch", str(t.dtype).replace("torch.", ""), list(t.shape), device, memoryview(raw)


def _strip(obj, path, found):
    """Copy of ``obj`` with every array replaced by None; ``found`` collects (path, array)."""
    if _is_device_result(obj):
        found.append(("result", path, None))
        return _strip(obj.wait(), path, found)
    if is_array(obj):
        found.append(("array", path, obj))
        return None
    if isinstance(obj, dict):
        return {k: _strip(v, path + [str(k)], found) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [_strip(v, path + [i], found) for i, v in enumerate(obj)]
    return obj


def encode_message(command: str, parameters, codec: str | None = None):
    """``generate(command, parameters)`` when nothing in ``parameters`` is an array, else the
    binary tensor payload (bytes)."""
    if parameters is None:
        parameters = []
    params = parameters if isinstance(parameters, dict) else list(parameters)
    if not has_arrays(params):
        return generate(command, params)
    found: list = []
    stripped = _strip(params, [], found)      # a dict keeps its keys: parse() returns a dict
    codec = codec or _CODEC
    entries, blobs, offset = [], [], 0
    results = []
    for what, path, value in found:
        if what == "result":
            results.append(path)
            continue
        kind, dtype, shape, device, raw = _host_bytes(value)
        data = zlib.compress(raw, 1) if codec == "zlib" else raw
        n = len(data) if codec == "zlib" else raw.nbytes
        entries.append({"path": path, "kind": kind, "dtype": dtype, "shape": shape, "device": device,
                        "offset": offset, "nbytes": n, "codec": codec})
        blobs.append(data)
        pad = (-n) % _ALIGN
        if pad:
            blobs.append(b"\x00" * pad)
        offset += n + pad
    header = json.dumps({"v": 1, "sexpr": generate(command, stripped), "arrays": entries,
                         "results": results}, separators=(",", ":")).encode()
    lead = len(MAGIC) + 4 + len(header)
    head_pad = (-lead) % _ALIGN
    return b"".join([MAGIC, struct.pack("<I", len(header)), header, b"\x00" * head_pad, *blobs])


_MAX_ARRAY_BYTES = 1 << 34                    # 16 GiB: far above any MQTT-borne array

_TORCH_DTYPES = ("float32", "float16", "bfloat16", "float64", "uint8", "int8", "int16", "int32", "int64",
                 "bool", "complex64", "complex128", "float8_e4m3fn", "float8_e5m2", "uint16", "uint32",
                 "uint64")


def _restore(entry, buf: memoryview, base: int):
    start = base + int(entry["offset"])
    n = int(entry["nbytes"])
    if start < base or start + n > len(buf):
        raise ValueError("tensor payload: blob outside the message")
    raw = buf[start:start + n]
    shape = [int(s) for s in entry["shape"]]
    if any(d < 0 for d in shape):
        raise ValueError("tensor payload: negative dimension")
    count = math.prod(shape)
    kind = entry["kind"]
    if kind == "numpy":
        np_dtype = np.dtype(entry["dtype"])
        if np_dtype.hasobject:
            raise ValueError("tensor payload: object dtype refused")
        itemsize = np_dtype.itemsize
    elif kind == "torch":
        import torch
        name = entry["dtype"]
        if name not in _TORCH_DTYPES:
            raise ValueError(f"tensor payload: dtype {name!r} refused")
        t_dtype = getattr(torch, name)
        itemsize = torch.empty((), dtype=t_dtype).element_size()
    else:
        raise ValueError(f"tensor payload: unknown array kind {kind!r}")
    expected = count * itemsize
    if expected > _MAX_ARRAY_BYTES:
        raise ValueError(f"tensor payload: {expected} bytes claimed for one array")
    codec = entry.get("codec", "raw")
    if codec == "zlib":
        # bounded: a blob may not inflate past the array it claims to be
        d = zlib.decompressobj()
        out = d.decompress(raw, expected + 1)
        raw = memoryview(out)
    elif codec != "raw":
        raise ValueError(f"tensor payload: unknown codec {codec!r}")
    if raw.nbytes != expected:
        raise ValueError(f"tensor payload: {raw.nbytes} bytes for a {entry['dtype']} array of shape {shape}")
    if kind == "numpy":
        return np.frombuffer(raw, dtype=np_dtype).reshape(shape).copy()
    dtype = t_dtype
    if count == 0:
        t = torch.empty(shape, dtype=dtype)
    else:
        t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).view(dtype).reshape(shape)
    if str(entry.get("device", "cpu")).startswith("cuda") and torch.cuda.is_available():
        t = t.to(torch.device("cuda", torch.cuda.current_device()))
    return t


def _place(tree, path, value):
    node = tree
    for key in path[:-1]:
        node = node[key]
    node[path[-1]] = value


def _get(tree, path):
    node = tree
    for key in path:
        node = node[key]
    return node


def decode_message(payload):
    """Binary tensor payload -> ``(command, parameters)`` with the arrays restored."""
    from ..utils.sexpr import parse
    buf = memoryview(payload)
    if bytes(buf[:len(MAGIC)]) != MAGIC:
        raise ValueError("not a tensor payload")
    (hlen,) = struct.unpack_from("<I", buf, len(MAGIC))
    h0 = len(MAGIC) + 4
    header = json.loads(bytes(buf[h0:h0 + hlen]).decode("utf-8"))
    base = h0 + hlen
    base += (-base) % _ALIGN
    command, params = parse(header["sexpr"])
    tree = params if isinstance(params, dict) else list(params)
    for entry in header.get("arrays", []):
        _place(tree, entry["path"], _restore(entry, buf, base))
    results = header.get("results") or []
    if results and _torch() is not None:
        try:
            from ..gpu.element import DeviceResult
        except Exception:                       # a torch process without the GPU half
            DeviceResult = None
        if DeviceResult is not None:
            for path in sorted(results, key=len, reverse=True):
                _place(tree, path, DeviceResult(_get(tree, path), None))
    return command, tree
