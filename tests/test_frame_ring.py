"""Shared-memory frame ring (binary media by slot id instead of zlib(np.save) over MQTT)."""
import multiprocessing as mp
import uuid

import numpy as np

from aiko_services_amd.message.frame_ring import SharedFrameRing, is_ring_token


def _reader(token, q):
    out = SharedFrameRing.get(token)
    q.put(None if out is None else (out.shape, int(out.sum())))


def test_ring_roundtrip_across_processes():
    ring = SharedFrameRing(f"aiko_t_{uuid.uuid4().hex[:8]}", slots=4, slot_bytes=64 * 48 * 3, create=True)
    try:
        img = np.random.default_rng(0).integers(0, 256, (48, 64, 3), dtype=np.uint8)
        tok = ring.put(img)
        assert is_ring_token(tok) and is_ring_token(tok.encode()) and len(tok) < 80
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        p = ctx.Process(target=_reader, args=(tok, q))
        p.start()
        got = q.get(timeout=60)
        p.join(30)
        assert got == ((48, 64, 3), int(img.sum()))
        assert np.array_equal(SharedFrameRing.get(tok), img)
    finally:
        ring.close()


def test_lapped_slot_is_detected():
    ring = SharedFrameRing(f"aiko_t_{uuid.uuid4().hex[:8]}", slots=2, slot_bytes=1024, create=True)
    try:
        first = ring.put(np.arange(10, dtype=np.int32))
        ring.put(np.arange(10, dtype=np.int32) * 2)
        ring.put(np.arange(10, dtype=np.int32) * 3)       # reuses the first token's slot
        assert SharedFrameRing.get(first) is None
    finally:
        ring.close()


def test_robot_video_payload_modes(monkeypatch):
    from aiko_services_amd.examples.xgo_robot import xgo_robot as X
    img = np.full((8, 8, 3), 7, np.uint8)
    assert np.array_equal(X.video_frame(X.video_payload(img)), img)          # zlib(np.save) default
    monkeypatch.setenv("AIKO_FRAME_RING", "1")
    payload = X.video_payload(img)
    assert is_ring_token(payload) and len(payload) < 80
    assert np.array_equal(X.video_frame(payload), img)
    X._RING.close()
    X._RING = None


def test_restarted_writer_is_reattached():
    """A writer that restarts recreates its ring under the same name (new generation): a reader
    that cached the old mapping re-attaches instead of serving the old run's slots."""
    name = f"aiko_t_{uuid.uuid4().hex[:8]}"
    ring = SharedFrameRing(name, slots=2, slot_bytes=1024, create=True)
    old = ring.put(np.full(4, 1, np.int32))
    assert SharedFrameRing.get(old).tolist() == [1] * 4          # reader caches the mapping
    ring.close()
    ring = SharedFrameRing(name, slots=2, slot_bytes=1024, create=True)
    try:
        new = ring.put(np.full(4, 2, np.int32))                  # same slot / seq as ``old``
        assert new.split("/")[2:] == old.split("/")[2:] and new != old
        assert SharedFrameRing.get(new).tolist() == [2] * 4
        assert SharedFrameRing.get(old) is None                  # the old run's frame is gone
    finally:
        ring.close()
