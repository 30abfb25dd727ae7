"""Shared host frame ring: image / audio payloads by slot id instead of bytes over MQTT.

The reference moves binary media between processes by publishing ``zlib(np.save(array))`` on an
MQTT topic (``/root/reference/src/aiko_services/examples/xgo_robot/xgo_robot.py:320-324``,
``robot_control.py:239-245``): every frame is serialised, compressed, copied through the broker
and decompressed.  On one node the payload can instead stay in a ring of fixed-size slots in
POSIX shared memory (``multiprocessing.shared_memory``); the MQTT message carries only a token

    R@<ring name>/<slot>/<sequence>/<dtype>/<d0>x<d1>x...

and the reader copies (or views) the slot.  Each slot starts with a 64-byte header holding its
sequence number, written before and after the payload (seqlock): a reader that finds the two
differing, or not equal to the token's sequence, knows the writer has lapped the ring and drops
the frame instead of returning torn data.  GPU peers use the RCCL hop plane
(``parallel/hop.py``) instead.
"""
from __future__ import annotations

import struct
from multiprocessing import shared_memory

import numpy as np

__all__ = ["SharedFrameRing", "is_ring_token", "RING_TOKEN"]

RING_TOKEN = "R@"
_HDR = 64
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
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=16 + slots * (_HDR + slot_bytes))
            struct.pack_into("<qq", self.shm.buf, 0, slots, slot_bytes)
        else:
            self.shm = shared_memory.SharedMemory(name=name)
            try:        # a reader must not unlink the writer's ring when it exits (bpo-38119)
                from multiprocessing import resource_tracker
                resource_tracker.unregister(self.shm._name, "shared_memory")
            except Exception:
                pass
            slots, slot_bytes = struct.unpack_from("<qq", self.shm.buf, 0)
        self.slots, self.slot_bytes = int(slots), int(slot_bytes)
        self.owner = create
        self.seq = 0

    @classmethod
    def attach(cls, name: str) -> "SharedFrameRing":
        ring = cls._attached.get(name)
        if ring is None:
            ring = cls._attached[name] = cls(name)
        return ring

    def _base(self, slot: int) -> int:
        return 16 + slot * (_HDR + self.slot_bytes)

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
        return f"{RING_TOKEN}{self.name}/{slot}/{self.seq}/{a.dtype.name}/{shape}"

    @staticmethod
    def get(token, copy: bool = True):
        """The array a token names, or None when the writer has reused the slot since."""
        if isinstance(token, (bytes, bytearray)):
            token = token.decode()
        name, slot, seq, dtype, shape = token[len(RING_TOKEN):].split("/")
        ring = SharedFrameRing.attach(name)
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
