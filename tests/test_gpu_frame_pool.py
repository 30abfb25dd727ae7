"""FramePool on the hot path: GPU-aware release / back-pressure, frames
decoded into pool slots, hipGraphs captured on the slots (no per-frame input copy)."""
import queue

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_release_after_blocks_until_gpu_done(native):
    from aiko_services_amd.gpu.element import FramePool
    pool = FramePool(2, 1 << 20, device="cuda:0")
    a, b = pool.acquire(0), pool.acquire(0)
    assert {a, b} == {0, 1}
    assert pool.acquire(0) == -1                       # exhausted, nothing pending: no slot
    x = torch.randn(4096, 4096, device="cuda")
    for _ in range(20):                                # keep the GPU busy for a while
        x = torch.tanh(x @ x)
    pool.release_after(a)                              # gated by an event behind that work
    pool.release_after(b)
    s = pool.acquire(0)                                # waits for the oldest release (back-pressure)
    assert s == a and torch.cuda.current_stream().query() in (True, False)
    st = pool.stats()
    assert st["high_water"] == 2 and st["exhausted"] >= 1


def _pipeline(pool, on_exhausted="block", batch=8):
    import bench
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    d = bench.definition(batch, True, 224, 224)
    d["elements"][0]["parameters"].update(pool=pool, on_exhausted=on_exhausted)
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(d), None, None, "s", [], 0, None, 60,
                                     queue_response=q)
    return p, q


def test_frames_in_pool_slots_and_graphs_on_slots(native):
    p, q = _pipeline(pool=3)
    results = []
    for i in range(9):
        p.process_frame({"stream_id": "s", "frame_id": i}, {})
        info, out = q.get_nowait()
        assert info["state"] == 0
        results.append(out["topk"])
    for r in results:
        r.wait()
    src = p.get_element("SyntheticFrames")
    st = src.frame_pool.stats()
    assert st["acquired"] == 3 + 9 and st["high_water"] <= 3     # 3 fills + 9 frames
    resnet = p.get_element("ResNet50Classifier")
    # per-address graphs live in the ("graphs", key, lane) LRU; the copy-in fallback is keyed
    # (key, lane) and must never have been created
    per_addr = [a for k, g in resnet._captured.items() if isinstance(k, tuple) and k[:1] == ("graphs",)
                for a in g]
    assert len(per_addr) == 3, per_addr                # one graph per slot address
    copy_in = [k for k in resnet._captured if isinstance(k, tuple) and len(k) == 2 and k[0] not in ("graphs", "seen")]
    assert not copy_in, copy_in                        # no copy path
    # same slot -> same frames -> same top-5 (frames 0, 3, 6 used slot 0)
    a, b = results[0].wait(), results[3].wait()
    assert torch.equal(a["top_index"], b["top_index"])


def test_exhausted_pool_drops_frames(native):
    """on_exhausted: drop — with the only slot still held by an unfinished frame the next
    frame is dropped (DROP_FRAME) instead of waiting."""
    from aiko_services_amd.pipeline.stream import Frame
    p, q = _pipeline(pool=1, on_exhausted="drop")
    src = p.get_element("SyntheticFrames")
    frame = Frame()                                    # a frame that has not completed yet
    p.create_stream("held", queue_response=queue.Queue())
    p._enable_thread_local("t", "held")
    p.stream_leases["held"].stream.frames[p.thread_local.frame_id] = frame
    try:
        ev, out = src.process_frame(None)
        assert ev == 0 and out["images"].shape == (8, 224, 224, 3)
        ev2, out2 = src.process_frame(None)
        assert ev2 == 1 and src.dropped == 1           # StreamEvent.DROP_FRAME
    finally:
        p._disable_thread_local("t")
    for cb in frame.on_complete:                       # the held frame completes
        cb()
    torch.cuda.synchronize()
    p.process_frame({"stream_id": "s", "frame_id": 0}, {})
    info, _ = q.get_nowait()
    assert info["state"] == 0                          # slot back: frames flow again
