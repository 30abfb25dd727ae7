"""Cross-stream ordering of the hop send path (VERDICT r3 item 2 / ADVICE r3 high).

A frame's hop tensors are produced on its lane's HIP stream, but the engine may encode them
later from a different stream: a queued frame dispatched from ANOTHER frame's lane
(``_remote_done`` -> ``_drain_pending``) or from the event loop (``_hop_timer``), and a group's
responses flushed after the members' lane scopes closed (``_flush_responses``).  Each case here
produces a tensor on lane 0 behind a long ``torch.cuda._sleep`` (its buffer holds a sentinel
until then), sends it from lane 1 or from the default stream over the loopback link (the same
staging copy + ordering as an RCCL send), and checks the received bytes are the produced ones.
Before the fix every case received the sentinel."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SLEEP = 40_000_000            # GPU cycles (~20 ms): the copy would run long before the producer


@pytest.fixture()
def plane(monkeypatch):
    import os
    from aiko_services_amd.parallel import hop
    if os.environ.get("AIKO_HOP_NO_ORDER") == "1":
        # negative control (run by hand, expected to FAIL): the pre-fix behaviour, no ordering
        monkeypatch.setattr(hop.HopPlane, "_order_after", lambda self, events: None)
    p = hop.init_plane([(0, 0)], device=torch.device("cuda", torch.cuda.current_device()), depth=4)
    yield p
    torch.cuda.synchronize()
    hop.shutdown_plane()


def _late(plane, lane, shape, value, dtype=torch.bfloat16):
    """A tensor written on lane ``lane`` only after a long sleep (a sentinel before that), and
    the producer's ready event."""
    from aiko_services_amd.gpu.lanes import lane_scope
    dev = plane.device
    x = torch.full(shape, -7.0, device=dev, dtype=dtype)
    torch.cuda.synchronize()
    with lane_scope(lane, dev):
        torch.cuda._sleep(SLEEP)
        x.fill_(value)
        ev = plane.ready_event()
    return x, ev


def _recv(plane, msg):
    got, handle = plane.decode(msg, pooled=True)
    out = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in got.items()}
    plane.release([handle])
    return out


def _recv_group(plane, msgs):
    outs, handle, work = plane.decode_group_async(msgs, pooled=True)
    assert work is None
    res = [{k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in o.items()} for o in outs]
    plane.release([handle] * len(msgs))
    return res


def test_single_hop_from_another_lane(plane):
    from aiko_services_amd.gpu.lanes import lane_scope
    x, ev = _late(plane, 0, (3, 224, 224), 5.0)
    with lane_scope(1, plane.device):                 # another frame's lane drains the queue
        msg = plane.encode(0, {"x": x, "n": 1}, key=("s", 1), ready=[ev])
    got = _recv(plane, msg)
    plane.ack(("s", 1))
    assert torch.equal(got["x"], x) and bool((got["x"] == 5.0).all())


def test_queued_frame_from_event_loop_after_producer_reuses_buffer(plane):
    """The engine's queue path: inputs captured on the producing lane (hold_inputs), the
    producer then rewrites its buffer for its next frame, and the event-loop thread (default
    stream) dispatches the queued frame."""
    from aiko_services_amd.gpu.lanes import lane_scope
    dev = plane.device
    x = torch.full((4, 1000), -7.0, device=dev)
    torch.cuda.synchronize()
    with lane_scope(0, dev):
        torch.cuda._sleep(SLEEP)
        x.fill_(3.0)                                   # frame k's output
        held, ready = plane.hold_inputs({"x": x, "tag": "k"})
        torch.cuda._sleep(SLEEP)
        x.fill_(4.0)                                   # the same buffer, frame k + 1's output
    msg = plane.encode(0, held, key=("s", 2), ready=[ready])    # _hop_timer: no lane
    got = _recv(plane, msg)
    plane.ack(("s", 2))
    assert got["tag"] == "k" and bool((got["x"] == 3.0).all())


def test_group_of_frames_from_two_lanes(plane):
    a, ev_a = _late(plane, 0, (2, 64, 64), 1.0)
    b, ev_b = _late(plane, 1, (2, 64, 64), 2.0)
    msgs = plane.encode_group(0, [{"x": a}, {"x": b}], keys=[("s", 3), ("s", 4)], ready=[ev_a, ev_b])
    got = _recv_group(plane, msgs)
    plane.ack(("s", 3))
    plane.ack(("s", 4))
    assert bool((got[0]["x"] == 1.0).all()) and bool((got[1]["x"] == 2.0).all())


def test_response_flush_after_lane_scope(plane):
    """``_flush_responses``: each member's response carries the event recorded on its lane when
    it completed; DeviceResult values are ordered after their own event."""
    from aiko_services_amd.gpu.element import DeviceResult
    from aiko_services_amd.gpu.lanes import lane_scope
    dev = plane.device
    top, ev_top = _late(plane, 0, (8, 5), 9.0, dtype=torch.float32)
    idx = torch.zeros(8, 5, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with lane_scope(1, dev):
        torch.cuda._sleep(SLEEP)
        idx.fill_(11)
        ev_idx = torch.cuda.Event()
        ev_idx.record()
    responses = [{"top": top}, {"r": DeviceResult({"i": idx}, ev_idx, t_submit=1.0)}]
    msgs = plane.encode_group(0, responses, ready=[ev_top, None])     # default stream
    got = _recv_group(plane, msgs)
    assert bool((got[0]["top"] == 9.0).all())
    r = got[1]["r"]
    assert isinstance(r, DeviceResult) and bool((r.wait()["i"] == 11).all())
    # and a single response
    top2, ev2 = _late(plane, 0, (8, 5), 10.0, dtype=torch.float32)
    got2 = _recv(plane, plane.encode(0, {"top": top2}, ready=[ev2]))
    assert bool((got2["top"] == 10.0).all())


def test_resend_from_another_stream(plane):
    """A held frame re-sent (its replica died) from another stream: ordered after the staging
    copy of the original send."""
    from aiko_services_amd.gpu.lanes import lane_scope
    x, ev = _late(plane, 0, (16, 4096), 6.0)
    with lane_scope(0, plane.device):
        msg = plane.encode(0, {"x": x}, key=("s", 5), ready=[ev])
    _recv(plane, msg)                                  # the first delivery (loopback queue)
    with lane_scope(1, plane.device):
        msg2 = plane.resend(("s", 5), 0)
    got = _recv(plane, msg2)
    plane.ack(("s", 5))
    assert bool((got["x"] == 6.0).all())
