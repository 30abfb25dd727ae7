"""Data plane parallelism over RCCL/xGMI: process groups, DP fan-out/gather, PP stage hand-off."""
from . import dist  # noqa: F401
