"""Remote-hop data plane: frame metadata over MQTT, tensor payloads over RCCL (xGMI).

The reference moves a frame to a remote PipelineElement by publishing the whole ``inputs``
dict as an S-expression (``/root/reference/src/aiko_services/main/pipeline.py:1072-1090``)
and continues the parent graph when ``process_frame_response`` comes back
(``:975-1006``).  Device tensors cannot ride in an S-expression, so on the MI355X path the hop
is split in two planes:

* control plane (unchanged, MQTT): ``(process_frame (stream_id: s frame_id: f hop_rank: r)
  (images: T@0/17/0/uint8/256x224x224x3 ...))`` — every tensor replaced by a short token
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

Credits (back-pressure).  A link has ``depth`` staging slots.  A FORWARD hop (``encode(...,
key=frame)``) holds its slot until the frame's response comes back (``ack(key)``): the slot is
the link's credit, so a sender can never have more frames in flight toward a peer than the
peer's receive pool holds (``depth`` slots, the receiver's FramePool) — the engine only picks a
replica with :meth:`credit` left and queues the frame otherwise.  The held slot is also the
RETRANSMIT buffer: when the peer dies the same bytes are re-sent to a survivor (:meth:`resend`)
or materialised locally (:meth:`held_values`), whatever the producing element has since written
into its own buffers.  Responses (``key=None``) use the slots as a ring: a slot is reused once
its previous transfer completed (the current stream waits on it: no host block on RCCL).

Failure.  :meth:`mark_dead` (registrar ``remove`` / last will of the peer's process, or a
transport error) retires every link to and from that rank: pending transfers are dropped, never
waited on (an RCCL send to a dead rank never completes and a ``wait()`` on it would stall this
GPU's stream), the per-link communicators are aborted, their staging buffers are not reused, and
any later use raises :class:`StageFailure`.  A frame abandoned while its peer is ALIVE
(:meth:`drop`: hop timeout, stream destroyed) never makes a stream wait on its send either: a
transfer still in flight keeps its slot and credit — and, zero-copy, its producer's FramePool
slot (:class:`Dropped`) — until :meth:`poll_dropped` sees it complete or the peer is retired.

Python floats (``t_submit`` stamps) travel as ``F@<repr>`` tokens so they keep their type;
:class:`~aiko_services_amd.gpu.element.DeviceResult` values travel as a nested dict of tensor
tokens and are rebuilt (with a completion event) on the receiver.
"""
from __future__ import annotations

import datetime
import os
import time
import weakref
from collections import deque

import torch
import torch.distributed as tdist

from . import dist as D
from .hop_state import (FLOAT_TOKEN, RESULT_KEY, TOKEN, NoCredit, StageFailure, is_token,  # noqa: F401
                        needs_decode, plane, set_plane)

__all__ = ["HopPlane", "Dropped", "StageFailure", "NoCredit", "init_plane", "plane", "shutdown_plane", "is_token",
           "needs_decode", "mark_frame_held", "TOKEN", "FLOAT_TOKEN"]

_ALIGN = 256
_DTYPES = {str(dt).split(".")[-1]: dt for dt in
           (torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.float16,
            torch.float32, torch.float64, torch.bfloat16, torch.bool)}
_DTYPE_NAMES = {dt: name for name, dt in _DTYPES.items()}


def _nbytes(dtype, shape) -> int:
    n = dtype.itemsize
    for d in shape:
        n *= int(d)
    return n


def _layout(specs):
    """Byte offsets of ``specs`` [(dtype, shape)] packed with 256-byte alignment; total size.
    A one-tensor message is exactly that tensor's bytes (it may be sent from the producer's
    own buffer, see :func:`mark_frame_held`)."""
    if len(specs) == 1:
        return [0], max(_nbytes(*specs[0]), 1)
    offs, at = [], 0
    for dt, shape in specs:
        offs.append(at)
        at += (_nbytes(dt, shape) + _ALIGN - 1) // _ALIGN * _ALIGN
    return offs, max(at, _ALIGN)


# Tensors whose storage their frame holds until it completes (a FramePool slot released by the
# frame's on_complete): a forward hop of such a tensor, alone in its message, is sent straight
# from it — no staging copy — since the frame (and so the buffer) outlives the hop's credit.
_FRAME_HELD: dict = {}


def mark_frame_held(t: torch.Tensor) -> torch.Tensor:
    """Declare that ``t``'s storage stays untouched until the current frame completes."""
    key = id(t)
    _FRAME_HELD[key] = weakref.ref(t, lambda _r, k=key: _FRAME_HELD.pop(k, None))
    return t


def _frame_held(t) -> bool:
    r = _FRAME_HELD.get(id(t))
    return r is not None and r() is t


def _view(buf: torch.Tensor, off: int, dtype, shape) -> torch.Tensor:
    n = _nbytes(dtype, shape)
    return buf[off:off + n].view(dtype).view(shape)


def _views(buf: torch.Tensor, offs, specs) -> list:
    """Typed views of ``specs`` [(dtype, shape)] at byte offsets ``offs`` of the uint8 buffer:
    one ``view(dtype)`` per distinct dtype + one ``as_strided`` per tensor (the offsets are
    256-byte aligned), instead of slice + two views per tensor."""
    typed = {}
    out = []
    nbytes = buf.numel()
    for off, (dt, shape) in zip(offs, specs):
        size = dt.itemsize
        if nbytes % size:
            out.append(_view(buf, off, dt, shape))
            continue
        base = typed.get(dt)
        if base is None:
            base = typed[dt] = buf.view(dt)
        stride, acc = [], 1
        for d in reversed(shape):
            stride.append(acc)
            acc *= d
        out.append(base.as_strided(shape, tuple(reversed(stride)), base.storage_offset() + off // size))
    return out


def _parse(tok: str):
    src, seq, idx, dt, shape = tok[len(TOKEN):].split("/")
    dims = tuple(int(s) for s in shape.split("x")) if shape else ()
    return int(src), int(seq), int(idx), _DTYPES[dt], dims


def _retoken(values: dict, seq: int) -> dict:
    """The token dict of a message with its per-link sequence number replaced."""
    out = {}
    for k, v in values.items():
        if isinstance(v, str) and v.startswith(TOKEN):
            f = v[len(TOKEN):].split("/")
            f[1] = str(seq)
            out[k] = TOKEN + "/".join(f)
        elif isinstance(v, dict):
            out[k] = _retoken(v, seq)
        else:
            out[k] = v
    return out


class _SendLink:
    """This rank -> ``peer``: process group + ``depth`` staging slots (credits)."""

    def __init__(self, peer, group, device, depth, grank=0):
        self.peer, self.group, self.device = peer, group, device
        self.grank = grank                  # the peer's rank within the link's 2-rank group
        self.bufs = [None] * depth
        self.work = [None] * depth          # last transfer that read the slot's buffer
        self.holder = [None] * depth        # frame key holding the slot until its ack
        self.free = depth                   # slots with no holder (the link's credits)
        self.cursor = 0
        self.seq = 0
        self.dead = False

    def credit(self) -> int:
        return 0 if self.dead else self.free

    def take(self, nbytes, key, staging=True):
        if self.dead:
            raise StageFailure(self.peer)
        n = len(self.bufs)
        for step in range(n):
            slot = (self.cursor + step) % n
            if self.holder[slot] is None:
                break
        else:
            raise NoCredit(f"hop: no credit toward rank {self.peer} ({n} frames unacknowledged)")
        self.cursor = (slot + 1) % n
        w = self.work[slot]
        if w is not None:
            w.wait()                         # RCCL: stream-ordered; gloo: host waits (CPU tests)
            self.work[slot] = None
        buf = self.bufs[slot]
        if staging and (buf is None or buf.numel() < nbytes):
            buf = self.bufs[slot] = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.holder[slot] = key
        self.free -= 1
        return slot, buf

    def release(self, slot, reuse=True):
        if self.holder[slot] is not None:
            self.free += 1
        self.holder[slot] = None
        if not reuse:                        # a transfer that may never finish still owns it
            self.work[slot] = None
            self.bufs[slot] = None

    def pending(self, slot):
        """The slot's transfer if it may still be reading its buffer (None once it finished)."""
        w = self.work[slot]
        if w is None:
            return None
        try:
            done = w.is_completed()
        except Exception:                    # noqa: BLE001 — a failed transfer reads nothing more
            done = True
        return None if done else w

    def retire(self):
        """Dead peer: forget every pending transfer (never wait on them) and every buffer."""
        self.dead = True
        keys = [k for k in self.holder if k is not None]
        n = len(self.bufs)
        self.bufs, self.work, self.holder = [None] * n, [None] * n, [None] * n
        self.free = 0
        return keys

    def drain(self):
        if self.dead:
            return
        for i, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[i] = None


class _RecvLink:
    """``peer`` -> this rank: process group + FramePool of receive slots (the sender's credits)."""

    def __init__(self, peer, group, device, depth, grank=0):
        self.peer, self.group, self.device, self.depth = peer, group, device, depth
        self.grank = grank
        self.pool = None
        self.seq = 0
        self.dead = False

    def slot(self, nbytes, plane, timeout_s: float = 30.0):
        pool = self.pool
        if pool is None or pool.slot_bytes < nbytes:
            from ..gpu.element import FramePool
            # capacity 2 x depth >= the sender's credits; sized for the largest message so far
            # (x1.25 headroom for small changes); slots of a retired pool stay valid: their frames
            # hold a reference to it
            pool = self.pool = FramePool(2 * self.depth, int(nbytes * 1.25) // _ALIGN * _ALIGN + _ALIGN,
                                         device=self.device if self.device.type == "cuda" else "cpu")
        s = pool.acquire(0.0)            # retires finished releases; waits on the GPU if all held
        if s < 0:
            # only a sender exceeding its credits gets here: wait for a slot (bounded), never
            # fall back to the allocator
            plane.counters["pool_waits"] += 1
            s = pool.acquire(timeout_s)
            if s < 0:
                plane.counters["pool_overflow"] += 1
                raise RuntimeError(f"hop: receive pool from rank {self.peer} exhausted for {timeout_s}s "
                                   "(sender exceeded its credits)")
        return (pool, s), pool.view(s, (pool.slot_bytes,), torch.uint8)


class Dropped:
    """A dropped forward frame whose transfer may still be reading its bytes (the peer is alive
    but has not posted the matching receive — stopped, hung, or just slow).  Its send slot and
    credit stay taken, and — for a zero-copy send out of the producer's FramePool slot — the
    callbacks the frame's owner hands over (:meth:`then`) are held back too, until
    :meth:`HopPlane.poll_dropped` sees the transfer complete or :meth:`HopPlane.mark_dead`
    retires the peer.  No stream ever waits on the transfer."""
    __slots__ = ("peer", "link", "slot", "work", "callbacks", "done")

    def __init__(self, peer, link, slot, work, host: bool = False):
        self.peer, self.link, self.slot, self.work = peer, link, slot, work
        self.callbacks: list = []
        self.done = None
        if host:
            # gloo: a send's Work only reports completion through wait(), which blocks until
            # the peer receives — so a daemon thread waits and flags it (RCCL: is_completed()
            # queries the transfer's end event, no thread)
            import threading
            self.done = False

            def waiter():
                try:
                    work.wait()
                except Exception:            # noqa: BLE001 — failed or aborted: reads nothing more
                    pass
                self.done = True
            threading.Thread(target=waiter, daemon=True, name="hop-dropped").start()

    def completed(self) -> bool:
        if self.done is not None:
            return self.done
        return self.link.pending(self.slot) is None

    def then(self, fn) -> None:
        self.callbacks.append(fn)

    def _finish(self, reuse):
        if reuse and not self.link.dead:
            self.link.work[self.slot] = None
            self.link.release(self.slot, reuse=True)
        callbacks, self.callbacks = self.callbacks, []
        for fn in callbacks:
            fn()


class _SharedSlot:
    """A receive slot shared by the members of a group message: free after the last release."""
    __slots__ = ("pool", "slot", "count")

    def __init__(self, pool, slot, count):
        self.pool, self.slot, self.count = pool, slot, count


class HopPlane:
    """Per-process RCCL data plane of the remote hops (see module docstring).

    ``links``: [(src, dst), ...] in the same order on every rank (each becomes one process
    group; every rank must call this constructor, it is collective over the default group).
    ``depth``: staging slots = credits per forward link = half the receive pool.
    """

    def __init__(self, links, device=None, depth: int = 4, rejoin=None):
        """``rejoin``: ``{"store": TCPStore client, "epoch": k}`` for a restarted rank joining a
        running plan: no default-group collectives here; :meth:`connect_rejoin` then builds
        its links as fresh 2-rank groups, as the survivors do in :meth:`readmit_connect`."""
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
        self.dead: set = set()
        self.suspect: set = set()          # alive but unresponsive peers (see suspend)
        self._suspect_since: dict = {}     # rank -> monotonic time of suspension / last probe
        self._probes: dict = {}            # rank -> probe frames sent while suspect
        self._probe_inflight: set = set()  # suspect ranks with a probe frame outstanding
        # a suspension is bounded: after probe_after_s one PROBE frame is admitted (a peer that
        # owes nothing would otherwise never be heard from again); after max_probes unanswered
        # probes suspend() asks the caller to retire the peer (mark_dead -> supervised restart)
        self.probe_after_s = float(os.environ.get("AIKO_HOP_PROBE_S", 30.0))
        self.max_probes = int(os.environ.get("AIKO_HOP_MAX_PROBES", 2))
        self._held: dict = {}              # frame / group key -> record (see _encode_many)
        self._loop: deque = deque()        # loopback link (src == dst): staged buffers in order
        self._groups: dict = {}            # (src, dst) -> process group
        self._waits = None                 # finish_later queue (host transfers), thread on first use
        self._member_of: dict = {}         # frame key -> group key (encode_group)
        self._group_seq = 0
        self._rejoin = rejoin
        self._readmit_callbacks: list = []  # fn(rank) after a restarted peer's links are back
        self.epochs: dict = {}             # peer rank -> epoch of its current links (0: original)
        self._rejoined: dict = {}          # peer rank -> epoch it announced all links up at
        self.counters = {"sent_msgs": 0, "sent_bytes": 0, "recv_msgs": 0, "recv_bytes": 0,
                         "pool_overflow": 0, "pool_waits": 0, "resent": 0, "dead_peers": 0, "zero_copy": 0,
                         "readmitted": 0, "dropped_inflight": 0, "dropped_completed": 0,
                         "suspended": 0, "probes": 0, "escalated": 0}
        self._dropped: list = []           # Dropped transfers still in flight (see drop)
        if rejoin is not None:
            for src, dst in self.links:
                if src == dst == self.rank:
                    self.send_links[dst] = _SendLink(dst, None, self.device, self.depth)
                    self.recv_links[src] = _RecvLink(src, None, self.device, self.depth)
            self.control = None
            return
        for src, dst in self.links:
            if src == dst:
                if src == self.rank:
                    self.send_links[dst] = _SendLink(dst, None, self.device, self.depth)
                    self.recv_links[src] = _RecvLink(src, None, self.device, self.depth)
                continue
            members = sorted({src, dst})
            group = tdist.new_group(ranks=members) if D.is_initialized() else None
            self._groups[(src, dst)] = group
            if src == self.rank:
                self.send_links[dst] = _SendLink(dst, group, self.device, self.depth, members.index(dst))
            elif dst == self.rank:
                self.recv_links[src] = _RecvLink(src, group, self.device, self.depth, members.index(src))
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

    # ---- re-admission of a restarted peer -----------------------------------------------------
    def _pair_links(self, peer: int, store, epoch: int, timeout_s: float):
        """Fresh 2-rank groups for every plan link between this rank and ``peer`` (a
        ``PrefixStore`` per link and epoch on the running group's store), brought up with the
        same one-element exchange as at start-up, in plan order on both sides.  Blocking."""
        from torch.distributed import PrefixStore
        backend = D.backend() or ("nccl" if self.device.type == "cuda" else "gloo")
        timeout = datetime.timedelta(seconds=timeout_s)
        send, recv, groups = {}, {}, {}
        for src, dst in self.links:
            if src == dst or {src, dst} != {self.rank, peer}:
                continue
            members = sorted({src, dst})
            ps = PrefixStore(f"aiko/hop/epoch{epoch}/{src}-{dst}", store)
            me = members.index(self.rank)
            if backend == "nccl":
                group = tdist.ProcessGroupNCCL(ps, me, 2, timeout)
            else:
                group = tdist.ProcessGroupGloo(ps, me, 2, timeout)
            groups[(src, dst)] = group
            other = members.index(peer)
            t = torch.zeros(1, dtype=torch.int64, device=self.device)
            if src == self.rank:
                send[dst] = _SendLink(dst, group, self.device, self.depth, other)
                group.send([t], other, 0).wait()
            else:
                recv[src] = _RecvLink(src, group, self.device, self.depth, other)
                group.recv([t], other, 0).wait()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        return {"peer": peer, "epoch": epoch, "send": send, "recv": recv, "groups": groups}

    def connect_rejoin(self, timeout_s: float = 120.0) -> list:
        """Restarted rank: bring up its links to every peer (each survivor does its side in
        :meth:`readmit_connect` once it hears the rejoin announcement).  Blocking; returns
        the peers connected."""
        if self._rejoin is None:
            raise RuntimeError("hop: connect_rejoin on a plane that did not start in rejoin mode")
        peers = []
        for src, dst in self.links:
            for peer in (src, dst):
                if peer != self.rank and self.rank in (src, dst) and peer not in peers:
                    peers.append(peer)
        for peer in peers:
            self.readmit_install(self._pair_links(peer, self._rejoin["store"], self._rejoin["epoch"], timeout_s))
        return peers

    def links_with(self, rank: int) -> bool:
        return any(self.rank in (s, d) and int(rank) in (s, d) and s != d for s, d in self.links)

    def readmit_connect(self, rank: int, epoch: int, timeout_s: float = 120.0):
        """Survivor side of a restarted peer's links, on the running group's store (blocking:
        run it off the actor thread, then :meth:`readmit_install` on it)."""
        from .rendezvous import group_store
        store = group_store()              # the raw TCPStore the restarted rank connects to
        if store is None:
            from torch.distributed.distributed_c10d import _get_default_store
            store = _get_default_store()
        return self._pair_links(int(rank), store, int(epoch), timeout_s)

    def readmit_install(self, pending) -> None:
        """Swap in a peer's fresh links (credits full, sequence numbers 0) and forget that it
        was dead.  The listeners (the engine re-adds the peer's replica) hear of it once the
        restarted peer has ALSO announced that every one of its links is up
        (:meth:`mark_rejoined`) — a middle stage must reach its downstream peers before it is
        given frames.  On the restarted rank itself they hear of it at once."""
        peer = pending["peer"]
        self.send_links.update(pending["send"])
        self.recv_links.update(pending["recv"])
        self._groups.update(pending["groups"])
        self.epochs[peer] = pending["epoch"]
        self._alive(peer)
        if peer in self.dead:
            self.dead.discard(peer)
            self.counters["readmitted"] += 1
        if self._rejoin is not None:
            self._notify_readmit(peer)
        elif self._rejoined.get(peer) == pending["epoch"]:
            self._notify_readmit(peer)

    def mark_rejoined(self, peer: int, epoch: int) -> None:
        """The restarted ``peer`` (at ``epoch``) has every link of the plan up again."""
        peer, epoch = int(peer), int(epoch)
        self._rejoined[peer] = epoch
        if self.epochs.get(peer) == epoch and peer not in self.dead:
            self._notify_readmit(peer)

    def _notify_readmit(self, peer) -> None:
        for fn in list(self._readmit_callbacks):
            fn(peer)

    def on_readmit(self, fn) -> None:
        self._readmit_callbacks.append(fn)

    # ---- credits / failure ------------------------------------------------------------------
    def credit(self, dst: int) -> int:
        """Frames that may still be sent toward ``dst`` before one is acknowledged."""
        dst = int(dst)
        link = self.send_links.get(dst)
        if link is None:
            return 0
        if dst in self.suspect:
            return min(1, link.credit()) if self._probe_due(dst) else 0
        return link.credit()

    def _probe_due(self, rank: int) -> bool:
        return rank not in self._probe_inflight and \
            time.monotonic() - self._suspect_since.get(rank, 0.0) >= self.probe_after_s

    def suspend(self, rank: int) -> bool:
        """A hop to ``rank`` timed out although the peer is not known dead (stopped, hung,
        overloaded): it gets no credit — no new frames — until it shows life again: a message
        from it arrives (:meth:`mark_alive`) or it is re-admitted.  The suspension is bounded:
        every ``probe_after_s`` one probe frame is let through (:meth:`credit`); returns True
        when ``max_probes`` probes went unanswered — the caller then retires the peer."""
        rank = int(rank)
        if rank == self.rank or rank in self.dead:
            return False
        if rank not in self.suspect:
            self.suspect.add(rank)
            self._suspect_since[rank] = time.monotonic()
            self._probes[rank] = 0
            self.counters["suspended"] += 1
            return False
        if rank in self._probe_inflight:          # the probe timed out too
            self._probe_inflight.discard(rank)
            self._suspect_since[rank] = time.monotonic()
            if self._probes.get(rank, 0) >= self.max_probes:
                self.counters["escalated"] += 1
                return True
        return False

    def _note_send(self, dst: int) -> None:
        """A frame (or group) is leaving toward ``dst``: while ``dst`` is suspect it is a probe."""
        if dst in self.suspect and dst not in self._probe_inflight:
            self._probe_inflight.add(dst)
            self._probes[dst] = self._probes.get(dst, 0) + 1
            self._suspect_since[dst] = time.monotonic()
            self.counters["probes"] += 1

    def mark_alive(self, rank: int) -> None:
        """``rank`` sent something (a message, a response): it is not stuck."""
        if self.suspect:
            rank = int(rank)
            self.suspect.discard(rank)
            self._probe_inflight.discard(rank)
            self._suspect_since.pop(rank, None)
            self._probes.pop(rank, None)

    _alive = mark_alive

    def is_dead(self, rank: int) -> bool:
        return int(rank) in self.dead

    def grouped(self, key) -> bool:
        """Whether held forward frame ``key`` travelled in a group message (:meth:`encode_group`)."""
        return key in self._member_of

    def ack(self, key) -> bool:
        """The response of forward frame ``key`` arrived: its staging slot is a credit again
        (a group's slot once every member is acknowledged or dropped).  True if a credit
        returned."""
        return self._settle(key, reuse=True)[0]

    def drop(self, key):
        """Abandon forward frame ``key`` (ERROR / timeout / stream destroyed).  A transfer that
        has finished gives its slot and credit back at once.  One that may still be reading
        (the peer never posted its receive) keeps both until it completes or the peer is
        retired (:meth:`poll_dropped`, :meth:`mark_dead`) — nothing waits on it.  Returns the
        :class:`Dropped` handle when the frame was sent zero-copy out of its producer's buffer
        and the caller must hold that buffer back (``handle.then(release)``); else None."""
        return self._settle(key, reuse=False)[1]

    def _settle(self, key, reuse):
        """-> (credit returned, Dropped handle of a zero-copy send still in flight or None)."""
        gk = self._member_of.pop(key, None)
        if gk is not None:
            rec = self._held.get(gk)
            if rec is None:
                return False, None
            members = rec[6]
            members.pop(key, None)
            rec[7] = rec[7] and reuse
            if members:
                return False, None
            key, reuse = gk, rec[7]
        rec = self._held.pop(key, None)
        if rec is None:
            return False, None
        link = self.send_links.get(rec[0])
        if link is None or link.dead or rec[1] is None:
            return False, None
        if not reuse:
            # RCCL: the end event says whether the transfer finished; gloo: only a wait can tell
            w = link.work[rec[1]] if self.host_transfers else link.pending(rec[1])
            if w is not None:
                # the transfer may outlive the frame: the slot (and, zero-copy, the producer's
                # buffer) stays taken until it completes — a stuck peer runs out of credits
                # instead of receiving more frames
                d = Dropped(rec[0], link, rec[1], w, host=self.host_transfers)
                self._dropped.append(d)
                self.counters["dropped_inflight"] += 1
                return False, (d if rec[9] else None)
        link.release(rec[1], reuse=True)       # the transfer finished: slot reusable as is
        return True, None

    def poll_dropped(self) -> int:
        """Finish every dropped transfer that completed: its slot becomes a credit again and
        the held callbacks run (e.g. the producer's FramePool slot release).  Returns how many
        are still in flight.  Called from the engine's hop timer and on responses."""
        if not self._dropped:
            return 0
        still = []
        for d in self._dropped:
            if d.link.dead or d.completed():
                # (not proof of life: a receive the peer posted before it stopped completes too)
                d._finish(reuse=True)
                self.counters["dropped_completed"] += 1
            else:
                still.append(d)
        self._dropped = still
        return len(still)

    @property
    def dropped_inflight(self) -> int:
        return len(self._dropped)

    def mark_dead(self, rank: int) -> list:
        """Retire every link to / from ``rank``; returns the keys of the forward frames it held
        (for :meth:`resend` / :meth:`held_values`, which keep working: the buffers are kept)."""
        rank = int(rank)
        if rank in self.dead or rank == self.rank:
            return []
        self.dead.add(rank)
        self.counters["dead_peers"] += 1
        keys = []
        link = self.send_links.get(rank)
        if link is not None:
            for key, rec in self._held.items():
                if rec[0] == rank:
                    rec[1] = None           # no slot any more: the record alone owns the buffer
                    keys.extend(rec[6] if rec[6] is not None else (key,))
            link.retire()
        rlink = self.recv_links.get(rank)
        if rlink is not None:
            rlink.dead = True
        if D.backend() == "nccl":
            for (src, dst), group in self._groups.items():
                if rank in (src, dst) and group is not None:
                    try:                    # stop RCCL's proxy waiting on the dead peer
                        from torch.distributed.distributed_c10d import _abort_process_group
                        _abort_process_group(group)
                    except Exception:       # noqa: BLE001 — best effort
                        pass
        # dropped transfers toward it will never complete: their held callbacks run now (the
        # link is retired, so nothing is reused under an RCCL kernel that the abort stopped)
        keep = []
        for d in self._dropped:
            if d.peer == rank:
                d._finish(reuse=False)
            else:
                keep.append(d)
        self._dropped = keep
        return keys

    # ---- stream ordering -------------------------------------------------------------------
    def ready_event(self):
        """An event on the current HIP stream (None off-GPU): recorded where a frame's tensors
        were produced, it lets :meth:`encode` run from any other stream — another frame's lane,
        the event-loop thread — and still copy / send them only once they are written."""
        if self.device.type != "cuda":
            return None
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def _order_after(self, events) -> None:
        if self.device.type != "cuda":
            return
        cur = torch.cuda.current_stream(self.device)
        for ev in events:
            if ev is not None:
                cur.wait_event(ev)

    def hold_inputs(self, values: dict):
        """A frame's hop inputs made safe to send LATER from another stream (a frame waiting for
        a credit): device tensors that are not frame-held (:func:`mark_frame_held`) are copied
        into storage the queue owns — the producer may rewrite its buffer for its next frame —
        and DeviceResults' device tensors likewise once their event passed.  Returns (values,
        event after the copies) — the event goes to :meth:`encode` as ``ready``."""
        from ..gpu.element import DeviceResult
        if self.device.type != "cuda" or not isinstance(values, dict):
            return values, None
        cur = torch.cuda.current_stream(self.device)

        def own(t):
            return t.clone() if t.device.type == "cuda" and not _frame_held(t) else t

        out = {}
        for k, v in values.items():
            if isinstance(v, torch.Tensor):
                out[k] = own(v)
            elif isinstance(v, DeviceResult):
                if v.event is not None:
                    cur.wait_event(v.event)
                # host tensors (pinned HostRing sets) stay by reference: a set is reused only
                # once the DeviceResult carrying it is dropped, and the queue holds it
                out[k] = DeviceResult({n: own(t) if isinstance(t, torch.Tensor) else t for n, t in v.tensors.items()},
                                      v.event, t_submit=v.t_submit, meta=v.meta)
            else:
                out[k] = v
        return out, self.ready_event()

    # ---- encode (sender) -------------------------------------------------------------------
    def encode(self, dst: int, values: dict, key=None, ready=None) -> dict:
        """``values`` with every tensor / DeviceResult / float replaced by tokens; the tensors
        are packed and sent to ``dst``.  ``key`` (forward hops): hold the staging slot until
        :meth:`ack` (raises :class:`NoCredit` when none is free).  Non-tensor values pass
        through unchanged.  ``ready``: events of the streams that produced the tensors (see
        :meth:`ready_event`); the staging copy and the send are ordered after them and after
        every DeviceResult's own event.  Without them the tensors must come from the current
        stream."""
        return self._encode_many(dst, [values], key, ready)[0]

    def encode_group(self, dst: int, values_list, keys=None, ready=None) -> list:
        """Several messages (frames) toward ``dst`` in ONE transfer: one staging slot, one
        send, one per-link sequence number; returns one token dict per message.  ``keys``
        (forward hops, one per frame): the slot is ONE credit, held until every member is
        acknowledged or dropped — control-plane cost per frame falls with the group size."""
        if keys is None:
            return self._encode_many(dst, values_list, None, ready)
        gk = ("group", self._group_seq)
        self._group_seq += 1
        outs = self._encode_many(dst, values_list, gk, ready)
        rec = self._held.get(gk)
        if rec is not None:
            rec[6] = {k: i for i, k in enumerate(keys)}
            for k in keys:
                self._member_of[k] = gk
        return outs

    def _encode_many(self, dst, values_list, key, ready=None):
        from ..gpu.element import DeviceResult
        dst = int(dst)
        link = self.send_links.get(dst)
        if link is None:
            if dst in self.dead or (self.rank, dst) in self.links:
                # a plan link that is not up (yet): a restarted rank before its rejoin finished
                raise StageFailure(dst, "link not connected")
            raise RuntimeError(f"hop: no send link {self.rank} -> {dst} in this plan")
        self._note_send(dst)
        tensors = []
        events = list(ready or ())

        def tok(v):
            if isinstance(v, torch.Tensor):
                tensors.append(v)
                return None                          # filled in below (needs the seq/index)
            if isinstance(v, float):
                return FLOAT_TOKEN + repr(v)
            return v

        outs, slots = [], []
        for values in values_list:
            out = {}
            for k, v in values.items():
                if isinstance(v, DeviceResult):
                    events.append(v.event)
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
            outs.append(out)
        if not tensors:
            return outs
        specs = [(t.dtype, tuple(t.shape)) for t in tensors]
        offs, total = _layout(specs)
        t0 = tensors[0]
        # zero copy: a forward hop whose only tensor is frame-held on this device goes out of
        # the producer's buffer (its credit still bounds the frames in flight)
        direct = (key is not None and len(tensors) == 1 and t0.device == self.device and t0.is_contiguous()
                  and dst != self.rank and _frame_held(t0))
        if dst == self.rank and key is None:
            # a loopback RESPONSE: the message owns its bytes (no ring slot, no credit — on the
            # loopback link the forward frames hold every credit of this same link object, and
            # in a multi-rank plan responses travel on the other direction's link)
            slot, buf = None, torch.empty(max(total, 1), dtype=torch.uint8, device=self.device)
        else:
            slot, buf = link.take(total, key if key is not None else (), staging=not direct)
        seq = link.seq
        link.seq += 1
        # the copy below and the send (RCCL's stream waits on the current one) read the tensors:
        # order the current stream after the streams that wrote them
        self._order_after(events)
        if direct:
            buf = t0.reshape(-1).view(torch.uint8)
            self.counters["zero_copy"] += 1
        else:
            for t, dstv in zip(tensors, _views(buf, offs, specs)):
                dstv.copy_(t if t.device == buf.device else t.to(buf.device, non_blocking=True),
                           non_blocking=True)
        for container, ckey, idx in slots:
            dt, shape = specs[idx]
            container[ckey] = (f"{TOKEN}{self.rank}/{seq}/{idx}/{_DTYPE_NAMES[dt]}/"
                               + "x".join(map(str, shape)))
        self._post(link, slot, buf, total, dst)
        if key is not None:
            # [dst, slot, total, specs, templates, buf, members (groups), slot reusable,
            #  event after the staging copy (a re-send from another stream waits on it),
            #  sent straight from the producer's frame-held buffer]
            self._held[key] = [dst, slot, total, specs, outs, buf, None, True, self.ready_event(), direct]
        else:
            if slot is not None:
                link.release(slot)                   # ring slot: free once its transfer is done
        return outs

    def _post(self, link, slot, buf, total, dst):
        D._account("hop_send", total)
        if dst == self.rank:
            # loopback: the message's own copy of its bytes — the staging slot may be reused
            # (ring / ack) before the receiver decodes, so the queue must not alias it
            # (its event: the receiver's stream is ordered after this copy, as an RCCL receive is
            # after the send it matches)
            self._loop.append((buf[:total] if slot is None else buf[:total].clone(), self.ready_event()))
            if slot is not None:
                link.work[slot] = None
        else:
            # the link's process group directly: tdist.isend re-validates group and rank per call
            link.work[slot] = link.group.send([buf[:total]], link.grank, 0) if link.group is not None \
                else None
        self.counters["sent_msgs"] += 1
        self.counters["sent_bytes"] += total

    def resend(self, key, dst: int) -> dict:
        """Send held forward frame ``key`` (its original bytes) to ``dst`` instead; returns the
        message's new token dict.  The frame then holds a credit of ``dst``'s link."""
        rec = self._held.get(key)
        if rec is None:
            raise KeyError(f"hop: no held frame {key}")
        if rec[6] is not None:
            raise ValueError("hop: a group's frames are re-sent one by one (held_values + encode)")
        dst = int(dst)
        link = self.send_links.get(dst)
        if link is None:
            raise StageFailure(dst) if dst in self.dead else RuntimeError(f"hop: no send link to {dst}")
        self._note_send(dst)
        old_dst, old_slot, total, specs, templates, buf = rec[:6]
        old = self.send_links.get(old_dst)
        if old is not None and not old.dead and old_slot is not None:
            old.release(old_slot, reuse=False)        # the buffer moves with the frame
        # the record keeps the bytes (a staging buffer, or the producer's frame-held buffer);
        # the new link's slot is only the credit — it must never alias them
        slot, _ = link.take(0, key, staging=False)
        seq = link.seq
        link.seq += 1
        self._order_after([rec[8]])                   # the bytes were staged on another stream
        self._post(link, slot, buf, total, dst)
        out = _retoken(templates[0], seq)
        self._held[key] = [dst, slot, total, specs, [out], buf, None, True, rec[8], rec[9]]
        self.counters["resent"] += 1
        return out

    def held_values(self, key) -> dict:
        """The held forward frame ``key`` as tensors (views of its staging buffer), e.g. to run
        it on a local replica after its remote peer died.  The frame keeps its record until
        :meth:`ack` / :meth:`drop`."""
        index = 0
        gk = self._member_of.get(key)
        if gk is not None:
            rec = self._held[gk]
            index = rec[6][key]
        else:
            rec = self._held[key]
        _dst, _slot, total, specs, templates, buf = rec[:6]
        offs, _ = _layout(specs)
        self._order_after([rec[8]])                   # staged on another stream
        return self._materialize(templates[index], buf, offs)

    def _materialize(self, template, buf, offs):
        from ..gpu.element import DeviceResult
        out = {}
        for k, v in template.items():
            if isinstance(v, str) and v.startswith(TOKEN):
                _src, _seq, idx, dt, shape = _parse(v)
                out[k] = _view(buf, offs[idx], dt, shape)
            elif isinstance(v, str) and v.startswith(FLOAT_TOKEN):
                out[k] = float(v[len(FLOAT_TOKEN):])
            elif isinstance(v, dict) and RESULT_KEY in v:
                sub = self._materialize({kk: vv for kk, vv in v.items() if kk != RESULT_KEY}, buf, offs)
                t_submit = sub.pop("_t_submit", None)
                out[k] = DeviceResult(sub, None, t_submit=t_submit)
            else:
                out[k] = v
        return out

    # ---- decode (receiver) -----------------------------------------------------------------
    _parse = staticmethod(_parse)

    @property
    def host_transfers(self) -> bool:
        """Whether a receive blocks the host until its bytes arrived (gloo, CPU tensors) rather
        than only ordering the current HIP stream after it (RCCL)."""
        return self.device.type != "cuda"

    def decode(self, values: dict, pooled: bool = True):
        """Inverse of :meth:`encode`: posts the receive of the message's tensors and returns
        ``(values, handle)``; ``handle`` (or None) must be given to :meth:`release` once the
        frame no longer needs the tensors (forward hops, ``pooled=True``).  Raises
        :class:`StageFailure` for a message of a dead peer or a failed transfer."""
        out, handle, work = self.decode_async(values, pooled)
        if work is not None:
            self.finish(work, handle)
        return out, handle

    def finish(self, work, handle) -> None:
        """Wait for a receive posted by :meth:`decode_async` (RCCL: the current stream waits,
        the host does not; gloo: the host blocks), then complete the message's DeviceResults
        (their event follows the receive).  A transfer error releases the slot and raises
        :class:`StageFailure`."""
        try:
            work[0].wait()
        except RuntimeError as exc:
            self.complete(work, handle, exc)
        self.complete(work, handle, None)

    def complete(self, work, handle, error) -> None:
        """Second half of :meth:`finish` once the wait is over (on the actor's thread)."""
        _w, src, results = work
        if error is not None:
            if handle is not None:
                self.release([handle] * (handle.count if isinstance(handle, _SharedSlot) else 1))
            raise StageFailure(src, error) from error
        self._results(results)

    def finish_later(self, work, callback) -> None:
        """Host-blocking transfers (gloo): wait for ``work`` on the plane's waiter thread, then
        call ``callback(error)`` (None, or the transport's exception) from that thread; the
        callback hands over to the actor, which calls :meth:`complete`.  The actor keeps
        dispatching while the bytes of several messages are in flight at once."""
        q = self._waits
        if q is None:
            import queue
            import threading
            q = self._waits = queue.SimpleQueue()

            def waiter():
                while True:
                    item = q.get()
                    if item is None:
                        return
                    w, cb = item
                    try:
                        w[0].wait()
                        err = None
                    except RuntimeError as exc:
                        err = exc
                    cb(err)

            threading.Thread(target=waiter, name="hop-waiter", daemon=True).start()
        q.put((work, callback))

    def _results(self, results):
        from ..gpu.element import DeviceResult
        for out, result_keys in results:
            for k in result_keys:
                v = out[k]
                t_submit = v.pop("_t_submit", None)
                ev = None
                if self.device.type == "cuda":
                    ev = torch.cuda.Event()
                    ev.record()
                out[k] = DeviceResult(v, ev, t_submit=t_submit)

    def decode_async(self, values: dict, pooled: bool = True):
        """:meth:`decode` without waiting for the bytes: ``(values, handle, work)``, ``work``
        (None when nothing is in flight) goes to :meth:`finish` before the values are read.
        Receives are still POSTED in message order here, so a link stays in order however the
        waits are scheduled."""
        outs, handle, work = self._decode_many([values], pooled)
        return outs[0], handle, work

    def decode_group_async(self, values_list, pooled: bool = True):
        """:meth:`decode_async` of an :meth:`encode_group` message: ``(values_list, handle,
        work)``; ``handle`` is shared by the members (give it to :meth:`release` once per
        member: the slot returns after the last)."""
        return self._decode_many(values_list, pooled)

    def _decode_many(self, values_list, pooled):
        found = []                   # (container, key, src, seq, idx, dtype, shape)
        outs = []

        def scan(container_in, container_out):
            for k, v in container_in.items():
                if isinstance(v, str) and v.startswith(TOKEN):
                    container_out[k] = None
                    found.append((container_out, k) + _parse(v))
                elif isinstance(v, str) and v.startswith(FLOAT_TOKEN):
                    container_out[k] = float(v[len(FLOAT_TOKEN):])
                elif isinstance(v, dict) and v.get(RESULT_KEY) is not None:
                    sub = {}
                    scan({kk: vv for kk, vv in v.items() if kk != RESULT_KEY}, sub)
                    container_out[k] = sub
                else:
                    container_out[k] = v

        for values in values_list:
            out = {}
            scan(values, out)
            outs.append(out)
        if not found:
            return outs, None, None
        srcs = {f[2] for f in found}
        seqs = {f[3] for f in found}
        if len(srcs) != 1 or len(seqs) != 1:
            raise RuntimeError(f"hop: one message must come from one send (got {srcs} / {seqs})")
        src, seq = srcs.pop(), seqs.pop()
        if src in self.dead:
            raise StageFailure(src, "message of a retired peer")
        self._alive(src)
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
            if len(values_list) > 1:
                handle = _SharedSlot(handle[0], handle[1], len(values_list))
        else:
            handle, buf = None, torch.empty(total, dtype=torch.uint8, device=self.device)
        D._account("hop_recv", total)
        work = None
        if src == self.rank:
            data, ev = self._loop.popleft()
            self._order_after([ev])
            buf[:total].copy_(data[:total], non_blocking=True)
        elif link.group is not None:
            try:
                work = link.group.recv([buf[:total]], link.grank, 0)
            except RuntimeError as exc:
                if handle is not None:
                    self.release([handle])
                raise StageFailure(src, exc) from exc
        self.counters["recv_msgs"] += 1
        self.counters["recv_bytes"] += total
        for f, v in zip(found, _views(buf, offs, specs)):
            f[0][f[1]] = v
        # DeviceResults are rebuilt once the receive is ordered (their completion event follows it)
        results = [(out, [k for k, v in values.items() if isinstance(v, dict) and RESULT_KEY in v])
                   for out, values in zip(outs, values_list)]
        if work is None:
            self._results(results)
            return outs, handle, None
        return outs, handle, (work, src, results)

    # ---- slot release ------------------------------------------------------------------------
    def release(self, handles) -> None:
        """Return receive slots once the work queued so far on the current stream is done
        (``FramePool.release_after``: a HIP event gates the reuse)."""
        for h in handles or []:
            if h is None:
                continue
            if isinstance(h, _SharedSlot):
                h.count -= 1
                if h.count > 0:
                    continue
                h = (h.pool, h.slot)
            pool, slot = h
            pool.release_after(slot)

    def barrier(self):
        if self.control is not None:
            tdist.barrier(group=self.control)

    def stats(self) -> dict:
        s = dict(self.counters)
        s["held_frames"] = sum(1 if rec[6] is None else len(rec[6]) for rec in self._held.values())
        s["dropped_pending"] = len(self._dropped)
        for dst, link in self.send_links.items():
            s[f"credit_to_{dst}"] = link.credit()
        for src, link in self.recv_links.items():
            if link.pool is not None:
                s[f"pool_free_from_{src}"] = link.pool.free_count()
        if self.dead:
            s["dead"] = sorted(self.dead)
        if self.suspect:
            s["suspect"] = sorted(self.suspect)
        return s

    def close(self):
        if self._waits is not None:
            self._waits.put(None)
        for link in self.send_links.values():
            link.drain()
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


def init_plane(links, device=None, depth: int = 4, rejoin=None) -> HopPlane:
    p = HopPlane(links, device=device, depth=depth, rejoin=rejoin)
    set_plane(p)
    return p


def shutdown_plane():
    p = plane()
    if p is not None:
        p.close()
    set_plane(None)
