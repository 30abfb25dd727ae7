"""Shared host frame ring: image / audio payloads by slot id instead of bytes over MQTT.

The reference moves binary media between processes by publishing ``zlib(np.save(array))`` on an
MQTT topic (``/root/reference/src/aiko_services/examples/xgo_robot/xgo_robot.py:320-324``,
``robot_control.py:239-245``): every frame is serialised, compressed, copied through the broker
and decompressed.  On one node the payload can instead stay in a ring of fixed-size slots in
POSIX shared memory (``multiprocessing.shared_memory``); the MQTT message carries only a token

    R@<ring name>/<generation>/<slot>/<sequence>/<dtype>/<d0>x<d1>x...

and the reader copies (or views) the slot.  ``generation`` is a random id the writer stores in
the ring header when it creates the ring: a reader re-attaches when a token names another
generation (the writer restarted and recreated the ring under the same name), so it never
reads a stale unlinked mapping.  Each slot starts with a 64-byte header holding its
sequence number, written before and after the payload (seqlock): a reader that finds the two
differing, or not equal to the token's sequence, knows the writer has lapped the ring and drops
the frame instead of returning torn data.  GPU peers use the RCCL hop plane
(``parallel/hop.py``) instead.
"""
from __future__ import annotations

import os
import struct
from multiprocessing import shared_memory

import numpy as np

__all__ = ["SharedFrameRing", "is_ring_token", "RING_TOKEN"]

RING_TOKEN = "R@"
_HDR = 64
_RING_HDR = 24                 # slots, slot_bytes, generation
_DTYPES = {np.dtype(t).name: np.dtype(t) for t in
           (np.uint8, np.int8, np.int16, np.uint16, np.int32, np.int64, np.float16, np.float32, np.float64)}


def is_ring_token(payload) -> bool:
    if isinstance(payload, (bytes, bytearray)):
        return payload[:2] == RING_TOKEN.encode()
    return isinstance(payload, str) and payload.startswith(RING_TOKEN)


class SharedFrameRing:
    """``slots`` x ``slot_bytes`` ring in shared memory ``name``.  The creating process
    (``create=True``) writes with :meth:`put`; others attach by name and :meth:`get`."""

    _attached: dict = {}

    def __init__(self, name: str, slots: int = 8, slot_bytes: int = 1 << 20, create: bool = False):
        self.name = name
        if create:
            try:                                        # a stale ring of a dead writer
                old = shared_memory.SharedMemory(name=name)
                old.close()
                old.unlink()
            except FileNotFoundError:
                pass
            self.shm = shared_memory.SharedMemory(name=name, create=True,
                                                  size=_RING_HDR + slots * (_HDR + slot_bytes))
            generation = int.from_bytes(os.urandom(7), "little")
            struct.pack_into("<qqq", self.shm.buf, 0, slots, slot_bytes, generation)
        else:
            self.shm = shared_memory.SharedMemory(name=name)
            try:        # a reader must not unlink the writer's ring when it exits (bpo-38119)
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
            slots, slot_bytes, generation = struct.unpack_from("<qqq", self.shm.buf, 0)
        self.slots, self.slot_bytes, self.generation = int(slots), int(slot_bytes), int(generation)
        self.owner = create
        self.seq = 0

    @classmethod
    def attach(cls, name: str, generation: int | None = None) -> "SharedFrameRing":
        """The mapping of ring ``name`` (cached); re-attached when ``generation`` differs from
        the cached one's (the writer recreated the ring)."""
        ring = cls._attached.get(name)
        if ring is not None and generation is not None and ring.generation != generation:
            cls._attached.pop(name, None)
            try:
                ring.shm.close()
            except Exception:       # noqa: BLE001 — a view may still hold the old buffer
                pass
            ring = None
        if ring is None:
            ring = cls._attached[name] = cls(name)
        return ring

    def _base(self, slot: int) -> int:
        return _RING_HDR + slot * (_HDR + self.slot_bytes)

    def put(self, array) -> str:
        """Copy ``array`` into the next slot; returns the token to publish."""
        a = np.ascontiguousarray(array)
        if a.nbytes > self.slot_bytes:
            raise ValueError(f"frame of {a.nbytes} B exceeds the ring's {self.slot_bytes} B slots")
        self.seq += 1
        slot = self.seq % self.slots
        base = self._base(slot)
        buf = self.shm.buf
        struct.pack_into("<q", buf, base, -self.seq)                  # writing
        buf[base + _HDR:base + _HDR + a.nbytes] = a.view(np.uint8).reshape(-1)
        struct.pack_into("<qq", buf, base, self.seq, self.seq)       # done (seq, seq-after)
        shape = "x".join(str(int(d)) for d in a.shape)
        return f"{RING_TOKEN}{self.name}/{self.generation}/{slot}/{self.seq}/{a.dtype.name}/{shape}"

    @staticmethod
    def get(token, copy: bool = True):
        """The array a token names, or None when the writer has reused the slot since."""
        if isinstance(token, (bytes, bytearray)):
            token = token.decode()
        name, generation, slot, seq, dtype, shape = token[len(RING_TOKEN):].split("/")
        try:
            ring = SharedFrameRing.attach(name, int(generation))
        except FileNotFoundError:
            return None                 # the writer is gone
        if ring.generation != int(generation):
            return None                 # a newer ring than the token's: the frame is gone
        slot, seq = int(slot), int(seq)
        dims = tuple(int(d) for d in shape.split("x")) if shape else ()
        dt = _DTYPES[dtype]
        base = ring._base(slot)
        s0, _ = struct.unpack_from("<qq", ring.shm.buf, base)
        if s0 != seq:
            return None
        n = int(np.prod(dims)) * dt.itemsize
        view = np.frombuffer(ring.shm.buf, dtype=np.uint8, count=n, offset=base + _HDR).view(dt).reshape(dims)
        out = view.copy() if copy else view
        s1, s2 = struct.unpack_from("<qq", ring.shm.buf, base)
        return out if s1 == seq and s2 == seq else None

    def close(self):
        self.shm.close()
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass
