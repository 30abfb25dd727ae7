"""Distributed data plane: one process per MI355X, ``torch.distributed`` over RCCL/xGMI.

``init()`` reads RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT (torchrun) and
creates the process group — backend ``nccl`` (= RCCL on ROCm) when a GPU is visible, ``gloo``
otherwise (CPU tests).  The collectives used by the pipeline engines:

* ``broadcast`` — DP fan-out of a frame batch from the ingest rank;
* ``scatter_frames`` — DP fan-out where each rank needs only its 1/N of the batch
  (grouped P2P sends: the root drives all 7 xGMI links at once);
* ``all_gather_into`` — DP result gather (fixed-size padded tensors);
* ``send`` / ``recv`` / ``batch_p2p`` — PP stage hand-off of activations.

xGMI on MI355X is point-to-point (7 links per GPU), so fan-out/fan-in is issued as grouped
P2P (one transfer per link) rather than ring algorithms wherever only the root needs data.

Every call is accounted in per-operation counters (calls, bytes moved by this rank) —
``comm_stats()`` — which GPU elements publish in their EC share (``rccl_mb``, ``rccl_gbps``)
and the tracer records as counter tracks (SURVEY §5.1 "RCCL bytes/latency counters").
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as tdist

__all__ = ["init", "is_initialized", "world_size", "rank", "local_rank", "barrier", "broadcast",
           "all_gather_into", "send", "recv", "batch_p2p", "scatter_frames", "all_reduce_max",
           "destroy", "backend", "comm_stats", "comm_bytes_total", "reset_comm_stats"]

_backend = None
_comm: dict = {}          # op -> [calls, bytes]
_identity = None          # (rank, world) of a re-admitted rank: no default process group exists


def _account(op: str, nbytes: int):
    c = _comm.get(op)
    if c is None:
        c = _comm[op] = [0, 0]
    c[0] += 1
    c[1] += int(nbytes)
    from ..utils.trace import get_tracer
    tracer = get_tracer()
    if tracer is not None:
        tracer.counter("rccl_bytes", {op: c[1]})


def _nbytes(t: torch.Tensor) -> int:
    return t.numel() * t.element_size()


def comm_stats() -> dict:
    """{op: {"calls": n, "bytes": b}} for this rank since start / the last reset."""
    return {op: {"calls": c, "bytes": b} for op, (c, b) in _comm.items()}


def comm_bytes_total() -> int:
    return sum(b for _, b in _comm.values())


def reset_comm_stats():
    _comm.clear()


def is_initialized() -> bool:
    return tdist.is_available() and tdist.is_initialized()


def world_size() -> int:
    if _identity is not None:
        return _identity[1]
    return tdist.get_world_size() if is_initialized() else 1


def rank() -> int:
    if _identity is not None:
        return _identity[0]
    return tdist.get_rank() if is_initialized() else 0


def set_identity(rank_: int, world: int, backend_name: str) -> None:
    """A restarted rank re-admitted into a running plan (``parallel/launch.py`` supervisor): it
    cannot join the original default process group, so its rank / world / backend are set
    here and its hop links are fresh 2-rank groups (``HopPlane`` rejoin mode)."""
    global _identity, _backend
    _identity = (int(rank_), int(world))
    _backend = backend_name


def local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def backend():
    return _backend


def init(backend_name: str | None = None, timeout_s: float | None = None, force: bool = False) -> bool:
    """Initialise from the environment when WORLD_SIZE > 1 (or ``force``: a world of one,
    e.g. to exercise the RCCL code paths on a single GPU); returns True if distributed."""
    global _backend
    if is_initialized():
        return True
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1 and not force:
        return False
    os.environ.setdefault("WORLD_SIZE", str(ws))
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    from ..utils.configuration import get_gpu_configuration
    cfg = get_gpu_configuration()
    if backend_name is None:
        backend_name = cfg.comm_backend or ("nccl" if torch.cuda.is_available() else "gloo")
    if timeout_s is None:
        timeout_s = cfg.comm_timeout_s
    kwargs = {}
    if backend_name == "nccl":
        dev = torch.device("cuda", cfg.device_for_local_rank(local_rank()) % max(1, torch.cuda.device_count()))
        torch.cuda.set_device(dev)
        kwargs["device_id"] = dev
    tdist.init_process_group(backend=backend_name, timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    _backend = backend_name
    return True


def barrier():
    if is_initialized():
        if _backend == "nccl":
            tdist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            tdist.barrier()


def broadcast(t: torch.Tensor, src: int = 0):
    if is_initialized():
        _account("broadcast", _nbytes(t))
        tdist.broadcast(t, src)
    return t


def all_gather_into(out: torch.Tensor, t: torch.Tensor):
    """``out`` = concat over ranks of ``t`` along dim 0 (out has world*len(t) rows)."""
    if not is_initialized():
        out.copy_(t)
        return out
    _account("all_gather", _nbytes(out))
    tdist.all_gather_into_tensor(out, t.contiguous())
    return out


def all_reduce_max(t: torch.Tensor):
    if is_initialized():
        _account("all_reduce", _nbytes(t))
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return t


def send(t: torch.Tensor, dst: int):
    _account("send", _nbytes(t))
    tdist.send(t, dst)


def recv(t: torch.Tensor, src: int):
    _account("recv", _nbytes(t))
    tdist.recv(t, src)
    return t


def batch_p2p(ops):
    """``ops`` = [("send"|"recv", tensor, peer), ...] issued as one grouped launch."""
    if not ops:
        return []
    for kind, t, _ in ops:
        _account(kind, _nbytes(t))
    p2p = [tdist.P2POp(tdist.isend if kind == "send" else tdist.irecv, t, peer) for kind, t, peer in ops]
    return tdist.batch_isend_irecv(p2p)


def scatter_frames(full: torch.Tensor | None, mine: torch.Tensor, src: int = 0):
    """Root sends rank r the r-th 1/N slice of ``full``; every rank receives into ``mine``."""
    if not is_initialized():
        mine.copy_(full)
        return mine
    ws, r = world_size(), rank()
    n = mine.shape[0]
    if r == src:
        ops = []
        for peer in range(ws):
            part = full[peer * n:(peer + 1) * n]
            if peer == src:
                mine.copy_(part)
            else:
                ops.append(("send", part.contiguous(), peer))
        for w in batch_p2p(ops):
            w.wait()
    else:
        for w in batch_p2p([("recv", mine, src)]):
            w.wait()
    return mine


def destroy():
    global _backend
    if is_initialized():
        tdist.destroy_process_group()
    _backend = None
