"""Remote-hop data plane: frame metadata over MQTT, tensor payloads over RCCL (xGMI).

The reference moves a frame to a remote PipelineElement by publishing the whole ``inputs``
dict as an S-expression (``/root/reference/src/aiko_services/main/pipeline.py:1072-1090``)
and continues the parent graph when ``process_frame_response`` comes back
(``:975-1006``).  Device tensors cannot ride in an S-expression, so on the MI355X path the hop
is split in two planes:

* control plane (unchanged, MQTT): ``(process_frame (stream_id: s frame_id: f hop_rank: r)
  (images: T@0/17/0/uint8/256x480x640x3 ...))`` — every tensor replaced by a short token
  naming the sending rank, the per-link message number, the tensor's index in the message and
  its dtype / shape;
* data plane (RCCL point-to-point over xGMI): the sender packs all tensors of the message into
  ONE staging buffer (device-to-device copy, 256-byte aligned regions) and posts one ``isend``;
  the receiver, when the MQTT message arrives, posts the matching ``irecv`` into a
  :class:`~aiko_services_amd.gpu.element.FramePool` slot (forward hops) or a fresh buffer
  (responses) and hands views of it to its elements.

Every direction of every link has its own process group (RCCL communicator): a rank's sends
to a peer and its receives from that peer then never serialise on one communicator stream,
which would deadlock a pipeline that has frame k+1 in flight forward while frame k's response
travels back.  P2P ops within one direction match in issue order, and the control messages of
one direction arrive in publish order (one MQTT connection per process), so no tags are
needed; the per-link message number is checked on receipt.

Send staging buffers form a ring of ``depth`` per link; a buffer is reused only after the
transfer that last read it completed (the current stream waits on it: no host block on RCCL).
Forward receive slots come from a capacity-``2 * depth`` FramePool per link and are released
when the frame completes — gated by a HIP event recorded at completion, so a slot is never
rewritten while kernels of that frame may still read it.  Pool exhaustion (more frames in
flight than slots) falls back to an allocator buffer and is counted in ``stats()``.

Python floats (``t_submit`` stamps) travel as ``F@<repr>`` tokens so they keep their type;
:class:`~aiko_services_amd.gpu.element.DeviceResult` values travel as a nested dict of tensor
tokens and are rebuilt (with a completion event) on the receiver.
"""
from __future__ import annotations

from collections import deque

import torch
import torch.distributed as tdist

from . import dist as D

__all__ = ["HopPlane", "init_plane", "plane", "shutdown_plane", "is_token", "TOKEN", "FLOAT_TOKEN"]

TOKEN = "T@"
FLOAT_TOKEN = "F@"
RESULT_KEY = "_device_result"
_ALIGN = 256
_DTYPES = {str(dt).split(".")[-1]: dt for dt in
           (torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.float16,
            torch.float32, torch.float64, torch.bfloat16, torch.bool)}


def is_token(v) -> bool:
    return isinstance(v, str) and (v.startswith(TOKEN) or v.startswith(FLOAT_TOKEN))


def _nbytes(dtype, shape) -> int:
    n = torch.empty((), dtype=dtype).element_size()
    for d in shape:
        n *= int(d)
    return n


def _layout(specs):
    """Byte offsets of ``specs`` [(dtype, shape)] packed with 256-byte alignment; total size."""
    offs, at = [], 0
    for dt, shape in specs:
        offs.append(at)
        at += (_nbytes(dt, shape) + _ALIGN - 1) // _ALIGN * _ALIGN
    return offs, max(at, _ALIGN)


def _view(buf: torch.Tensor, off: int, dtype, shape) -> torch.Tensor:
    n = _nbytes(dtype, shape)
    return buf[off:off + n].view(dtype).view(shape)


class _SendLink:
    """This rank -> ``peer``: process group + ring of staging buffers."""

    def __init__(self, peer, group, device, depth):
        self.peer, self.group, self.device = peer, group, device
        self.bufs = [None] * depth
        self.pending = [None] * depth
        self.cursor = 0
        self.seq = 0

    def stage(self, nbytes):
        slot = self.cursor
        self.cursor = (slot + 1) % len(self.bufs)
        w = self.pending[slot]
        if w is not None:
            w.wait()                       # RCCL: stream-ordered; gloo: host waits (CPU tests)
            self.pending[slot] = None
        buf = self.bufs[slot]
        if buf is None or buf.numel() < nbytes:
            buf = self.bufs[slot] = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return slot, buf

    def drain(self):
        for i, w in enumerate(self.pending):
            if w is not None:
                w.wait()
                self.pending[i] = None


class _RecvLink:
    """``peer`` -> this rank: process group + FramePool of receive slots."""

    def __init__(self, peer, group, device, depth):
        self.peer, self.group, self.device, self.depth = peer, group, device, depth
        self.pool = None
        self.seq = 0

    def slot(self, nbytes, plane):
        pool = self.pool
        if pool is None or pool.slot_bytes < nbytes:
            from ..gpu.element import FramePool
            # slots sized for the largest message so far (x1.25 headroom for small changes);
            # slots of a retired pool stay valid: their frames hold a reference to it
            pool = self.pool = FramePool(2 * self.depth, int(nbytes * 1.25) // _ALIGN * _ALIGN + _ALIGN,
                                         device=self.device if self.device.type == "cuda" else "cpu")
        s = pool.acquire(0.0)          # retires finished releases; waits on the GPU if all held
        if s < 0:                      # more frames in flight than slots: allocator buffer
            plane.counters["pool_overflow"] += 1
            return None, torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        return (pool, s), pool.view(s, (pool.slot_bytes,), torch.uint8)


class HopPlane:
    """Per-process RCCL data plane of the remote hops (see module docstring).

    ``links``: [(src, dst), ...] in the same order on every rank (each becomes one process
    group; every rank must call this constructor, it is collective over the default group).
    """

    def __init__(self, links, device=None, depth: int = 4):
        self.rank = D.rank()
        self.world = D.world_size()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if D.backend() == "nccl" \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.depth = max(2, int(depth))
        self.send_links: dict = {}
        self.recv_links: dict = {}
        self.links = [tuple(int(x) for x in l) for l in links]
        self._loop: deque = deque()        # loopback link (src == dst): staged buffers in order
        for src, dst in self.links:
            if src == dst:
                if src == self.rank:
                    self.send_links[dst] = _SendLink(dst, None, self.device, self.depth)
                    self.recv_links[src] = _RecvLink(src, None, self.device, self.depth)
                continue
            group = tdist.new_group(ranks=sorted({src, dst})) if D.is_initialized() else None
            if src == self.rank:
                self.send_links[dst] = _SendLink(dst, group, self.device, self.depth)
            elif dst == self.rank:
                self.recv_links[src] = _RecvLink(src, group, self.device, self.depth)
        # Bring every link's communicator up now, in the same global order on every rank: RCCL
        # creates a P2P communicator lazily at the first send/recv and blocks until the peer
        # joins, but the peer only posts its receive once the frame's MQTT message arrives —
        # which is published after the send.  A tiny exchange per link here breaks that cycle.
        for src, dst in self.links:
            if self.rank not in (src, dst) or src == dst or not D.is_initialized():
                continue
            link = self.send_links.get(dst) if src == self.rank else self.recv_links.get(src)
            t = torch.zeros(1, dtype=torch.int64, device=self.device)
            if src == self.rank:
                tdist.isend(t, dst, group=link.group).wait()
            else:
                tdist.irecv(t, src, group=link.group).wait()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        # host-side control group (gloo) for start-up barriers issued from helper threads
        self.control = tdist.new_group(backend="gloo") if D.is_initialized() else None
        self.counters = {"sent_msgs": 0, "sent_bytes": 0, "recv_msgs": 0, "recv_bytes": 0,
                         "pool_overflow": 0}

    # ---- encode (sender) -------------------------------------------------------------------
    def encode(self, dst: int, values: dict) -> dict:
        """``values`` with every tensor / DeviceResult / float replaced by tokens; the tensors
        are packed and sent to ``dst``.  Non-tensor values pass through unchanged."""
        from ..gpu.element import DeviceResult
        link = self.send_links.get(int(dst))
        if link is None:
            raise RuntimeError(f"hop: no send link {self.rank} -> {dst} in this plan")
        tensors = []

        def tok(v):
            if isinstance(v, torch.Tensor):
                tensors.append(v)
                return None                          # filled in below (needs the seq/index)
            if isinstance(v, float):
                return FLOAT_TOKEN + repr(v)
            return v

        out, slots = {}, []
        for k, v in values.items():
            if isinstance(v, DeviceResult):
                d = {RESULT_KEY: "1"}
                t = v.t_submit
                if isinstance(t, torch.Tensor):
                    t = int(t.reshape(-1)[0]) * 1e-9
                if isinstance(t, float):
                    d["_t_submit"] = FLOAT_TOKEN + repr(t)
                for name, tv in v.tensors.items():
                    d[name] = tok(tv)
                    if d[name] is None:
                        slots.append((d, name, len(tensors) - 1))
                out[k] = d
            else:
                out[k] = tok(v)
                if out[k] is None:
                    slots.append((out, k, len(tensors) - 1))
        if not tensors:
            return out
        seq = link.seq
        link.seq += 1
        specs = [(t.dtype, tuple(t.shape)) for t in tensors]
        offs, total = _layout(specs)
        slot, buf = link.stage(total)
        for t, off, (dt, shape) in zip(tensors, offs, specs):
            dstv = _view(buf, off, dt, shape)
            dstv.copy_(t if t.device == buf.device else t.to(buf.device, non_blocking=True),
                       non_blocking=True)
        for container, key, idx in slots:
            dt, shape = specs[idx]
            container[key] = (f"{TOKEN}{self.rank}/{seq}/{idx}/{str(dt).split('.')[-1]}/"
                              + "x".join(str(int(s)) for s in shape))
        D._account("hop_send", total)
        if int(dst) == self.rank:               # loopback: the receiver copies from the stage
            self._loop.append(buf)
            link.pending[slot] = None
        else:
            link.pending[slot] = tdist.isend(buf[:total], dst, group=link.group) if link.group is not None \
                else None
        self.counters["sent_msgs"] += 1
        self.counters["sent_bytes"] += total
        return out

    # ---- decode (receiver) -----------------------------------------------------------------
    @staticmethod
    def _parse(tok: str):
        src, seq, idx, dt, shape = tok[len(TOKEN):].split("/")
        dims = tuple(int(s) for s in shape.split("x")) if shape else ()
        return int(src), int(seq), int(idx), _DTYPES[dt], dims

    def decode(self, values: dict, pooled: bool = True):
        """Inverse of :meth:`encode`: posts the receive of the message's tensors and returns
        ``(values, handle)``; ``handle`` (or None) must be given to :meth:`release` once the
        frame no longer needs the tensors (forward hops, ``pooled=True``)."""
        from ..gpu.element import DeviceResult
        found = []                   # (container, key, src, seq, idx, dtype, shape)
        out = {}

        def scan(container_in, container_out):
            for k, v in container_in.items():
                if isinstance(v, str) and v.startswith(TOKEN):
                    container_out[k] = None
                    found.append((container_out, k) + self._parse(v))
                elif isinstance(v, str) and v.startswith(FLOAT_TOKEN):
                    container_out[k] = float(v[len(FLOAT_TOKEN):])
                elif isinstance(v, dict) and v.get(RESULT_KEY) is not None:
                    sub = {}
                    scan({kk: vv for kk, vv in v.items() if kk != RESULT_KEY}, sub)
                    container_out[k] = sub
                else:
                    container_out[k] = v

        scan(values, out)
        if not found:
            return out, None
        srcs = {f[2] for f in found}
        seqs = {f[3] for f in found}
        if len(srcs) != 1 or len(seqs) != 1:
            raise RuntimeError(f"hop: one message must come from one send (got {srcs} / {seqs})")
        src, seq = srcs.pop(), seqs.pop()
        link = self.recv_links.get(src)
        if link is None:
            raise RuntimeError(f"hop: no receive link {src} -> {self.rank} in this plan")
        if seq != link.seq:
            raise RuntimeError(f"hop: message {seq} from rank {src} out of order (expected {link.seq})")
        link.seq += 1
        found.sort(key=lambda f: f[4])
        specs = [(f[5], f[6]) for f in found]
        offs, total = _layout(specs)
        if pooled:
            handle, buf = link.slot(total, self)
        else:
            handle, buf = None, torch.empty(total, dtype=torch.uint8, device=self.device)
        D._account("hop_recv", total)
        if src == self.rank:
            buf[:total].copy_(self._loop.popleft()[:total], non_blocking=True)
        elif link.group is not None:
            tdist.irecv(buf[:total], src, group=link.group).wait()    # RCCL: the stream waits
        self.counters["recv_msgs"] += 1
        self.counters["recv_bytes"] += total
        for f, off in zip(found, offs):
            container, key = f[0], f[1]
            container[key] = _view(buf, off, f[5], f[6])
        # rebuild DeviceResults: completion event after the receive on this stream
        for k, v in list(out.items()):
            if isinstance(v, dict) and isinstance(values.get(k), dict) and RESULT_KEY in values[k]:
                t_submit = v.pop("_t_submit", None)
                ev = None
                if self.device.type == "cuda":
                    ev = torch.cuda.Event()
                    ev.record()
                out[k] = DeviceResult(v, ev, t_submit=t_submit)
        return out, handle

    # ---- slot release ------------------------------------------------------------------------
    def release(self, handles) -> None:
        """Return receive slots once the work queued so far on the current stream is done
        (``FramePool.release_after``: a HIP event gates the reuse)."""
        for h in handles or []:
            if h is not None:
                pool, slot = h
                pool.release_after(slot)

    def barrier(self):
        if self.control is not None:
            tdist.barrier(group=self.control)

    def stats(self) -> dict:
        s = dict(self.counters)
        for src, link in self.recv_links.items():
            if link.pool is not None:
                s[f"pool_free_from_{src}"] = link.pool.free_count()
        return s

    def close(self):
        for link in self.send_links.values():
            link.drain()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


_plane: HopPlane | None = None


def init_plane(links, device=None, depth: int = 4) -> HopPlane:
    global _plane
    _plane = HopPlane(links, device=device, depth=depth)
    return _plane


def plane() -> HopPlane | None:
    return _plane


def shutdown_plane():
    global _plane
    if _plane is not None:
        _plane.close()
    _plane = None
