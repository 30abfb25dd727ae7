"""GPU pipeline path on MI355X: aiko Pipeline with device-resident elements, frame pool."""
import queue

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_resnet_pipeline_matches_direct_model(native):
    import bench
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    for graph in (False, True):
        d = parse_pipeline_definition_dict(bench.definition(4, graph, 224, 224))
        q = queue.Queue()
        p = PipelineImpl.create_pipeline("<t>", d, None, None, "g", [], 0, None, 60, queue_response=q)
        results = []
        for i in range(3):
            p.process_frame({"stream_id": "g", "frame_id": i}, {})
            info, out = q.get_nowait()
            assert info["state"] == 0
            results.append(out["topk"])
        frames = p.get_element("SyntheticFrames")._pool
        model = ResNet50(seed=0, device="cuda")
        for i, r in enumerate(results):
            got = r.wait()
            prob, idx = model(frames[i % len(frames)])
            torch.cuda.synchronize()
            assert torch.equal(got["top_index"], idx.cpu())
            assert torch.allclose(got["top_prob"], prob.cpu(), rtol=1e-4, atol=1e-6)
            assert r.latency is not None and r.latency > 0


def test_frame_pool_on_device(native):
    from aiko_services_amd.gpu.element import FramePool
    pool = FramePool(3, 224 * 224 * 3, device="cuda:0")
    slots = [pool.acquire(0.1) for _ in range(3)]
    assert sorted(slots) == [0, 1, 2] and pool.acquire(0.01) == -1
    v = pool.view(slots[0], (224, 224, 3), torch.uint8)
    assert v.is_cuda and v.shape == (224, 224, 3)
    v.fill_(7)
    w = pool.view(slots[0], (224 * 224 * 3,), torch.uint8)
    assert int(w.sum()) == 7 * 224 * 224 * 3
    pool.release(slots[1])
    assert pool.acquire(0.1) == slots[1]
    st = pool.stats()
    assert st["capacity"] == 3 and st["high_water"] == 3 and st["exhausted"] == 1
