"""Data plane parallelism over RCCL/xGMI: process groups, DP fan-out/gather, PP stage hand-off.

Submodules are imported on use (``from aiko_services_amd.parallel import dist``): ``dist`` and
``hop`` load torch, which control-plane processes must not pay for."""
import importlib


def __getattr__(name):
    if name in ("dist", "hop", "hop_state", "launch", "placement", "rendezvous"):
        return importlib.import_module(f"{__name__}.{name}")
    raise AttributeError(name)
