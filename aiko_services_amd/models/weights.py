"""Weight persistence for the inference models ("save/load_state_dict for element
weights and fp8 scale tables"; the reference has no computation checkpointing at all).

Models expose ``named_layers()`` -> (name, layer) pairs, where a layer is a packed ``ConvSpec``
(bf16 [Cout, K] + fp32 bias, folded BatchNorm), an ``Fp8Linear`` (e4m3 bytes [N, Kp] + fp32
per-channel scale table + bias) or a plain tensor / tuple of tensors (LayerNorm gamma, beta).
The state dict stores exactly what the kernels consume, so loading needs no re-packing or
re-quantisation and is bit-exact; files are safetensors (no pickle on load) with the model's
constructor config in the metadata.

The fp32 reference copies used by the numerics tests (``ref_weight``) are optional
(``with_reference=True``); loading a dict without them drops the stale references.
"""
from __future__ import annotations

import json

import torch

__all__ = ["state_dict", "load_state_dict", "save_weights", "load_weights", "read_metadata", "WeightsMixin"]


def _layer_tensors(layer, with_reference: bool):
    from ..ops.conv import ConvSpec
    from ..ops.transformer import Fp8Linear
    if isinstance(layer, ConvSpec):
        out = {"weight": layer.weight, "bias": layer.bias}
        if with_reference:
            out.update(ref_weight=layer.ref_weight, ref_bias=layer.ref_bias)
        return out
    if isinstance(layer, Fp8Linear):
        out = {"weight": layer.weight, "scale": layer.scale, "bias": layer.bias}
        if with_reference:
            out["ref_weight"] = layer.ref_weight
        return out
    if isinstance(layer, torch.Tensor):
        return {"": layer}
    if isinstance(layer, (tuple, list)):
        return {str(i): t for i, t in enumerate(layer)}
    raise TypeError(f"unsupported layer type {type(layer).__name__}")


def state_dict(model, with_reference: bool = False) -> dict:
    sd = {}
    for name, layer in model.named_layers():
        for k, t in _layer_tensors(layer, with_reference).items():
            if t is not None:
                sd[f"{name}.{k}" if k else name] = t.detach().cpu().contiguous()
    return sd


def load_state_dict(model, sd: dict, strict: bool = True) -> list:
    """Copy ``sd`` into the model's tensors in place (device buffers keep their addresses, so
    captured hipGraphs stay valid).  Returns the keys that were not found when ``strict=False``."""
    from ..ops.conv import ConvSpec
    from ..ops.transformer import Fp8Linear
    missing, used = [], set()
    for name, layer in model.named_layers():
        for k, t in _layer_tensors(layer, with_reference=False).items():
            if t is None:
                continue
            key = f"{name}.{k}" if k else name
            src = sd.get(key)
            if src is None:
                missing.append(key)
                continue
            if tuple(src.shape) != tuple(t.shape) or src.dtype != t.dtype:
                raise ValueError(f"load_state_dict: {key} is {src.dtype}{tuple(src.shape)}, "
                                 f"model expects {t.dtype}{tuple(t.shape)}")
            t.copy_(src.to(t.device))
            used.add(key)
        if isinstance(layer, (ConvSpec, Fp8Linear)):
            ref = sd.get(f"{name}.ref_weight")
            layer.ref_weight = None if ref is None else ref.to(layer.weight.device)
            used.add(f"{name}.ref_weight")
            if isinstance(layer, ConvSpec):
                rb = sd.get(f"{name}.ref_bias")
                layer.ref_bias = None if rb is None else rb.to(layer.weight.device)
                used.add(f"{name}.ref_bias")
    unexpected = [k for k in sd if k not in used]
    if strict and (missing or unexpected):
        raise KeyError(f"load_state_dict: missing {missing[:8]}, unexpected {unexpected[:8]}")
    on_load = getattr(model, "_weights_loaded", None)
    if on_load is not None:
        on_load()
    from ..ops.conv import refresh_derived
    for spec in _walk_specs(model, set(), 0):       # incl. fused specs outside named_layers
        refresh_derived(spec)
    return missing


def _walk_specs(obj, seen: set, depth: int):
    """Every ConvSpec reachable from ``obj`` through this package's objects, lists and dicts."""
    from ..ops.conv import ConvSpec
    if id(obj) in seen or depth > 5 or isinstance(obj, torch.Tensor):
        return
    seen.add(id(obj))
    if isinstance(obj, ConvSpec):
        yield obj
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            yield from _walk_specs(o, seen, depth + 1)
    elif isinstance(obj, dict):
        for o in obj.values():
            yield from _walk_specs(o, seen, depth + 1)
    elif type(obj).__module__.startswith("aiko_services_amd") and hasattr(obj, "__dict__"):
        for o in vars(obj).values():
            yield from _walk_specs(o, seen, depth + 1)


def save_weights(model, path: str, with_reference: bool = False) -> None:
    from safetensors.torch import save_file
    meta = {"format": "aiko_services_amd", "model": type(model).__name__,
            "config": json.dumps(getattr(model, "config", lambda: {})())}
    save_file(state_dict(model, with_reference), path, metadata=meta)


def read_metadata(path: str) -> dict:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = dict(f.metadata() or {})
    if "config" in meta:
        meta["config"] = json.loads(meta["config"])
    return meta


def load_weights(model, path: str, strict: bool = True) -> list:
    from safetensors.torch import load_file
    meta = read_metadata(path)
    if meta.get("model") not in (None, type(model).__name__):
        raise ValueError(f"{path} holds {meta['model']} weights, not {type(model).__name__}")
    return load_state_dict(model, load_file(path), strict)


class WeightsMixin:
    """``state_dict`` / ``load_state_dict`` / ``save`` / ``load`` for a model with ``named_layers``."""

    def state_dict(self, with_reference: bool = False) -> dict:
        return state_dict(self, with_reference)

    def load_state_dict(self, sd: dict, strict: bool = True) -> list:
        return load_state_dict(self, sd, strict)

    def save(self, path: str, with_reference: bool = False) -> None:
        save_weights(self, path, with_reference)

    def load(self, path: str, strict: bool = True) -> list:
        return load_weights(self, path, strict)
