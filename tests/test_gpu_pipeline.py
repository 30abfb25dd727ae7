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
    for graph, lanes in ((False, 1), (True, 1), (True, 2), (False, 3)):
        d = parse_pipeline_definition_dict(bench.definition(4, graph, 224, 224, lanes))
        q = queue.Queue()
        p = PipelineImpl.create_pipeline("<t>", d, None, None, "g", [], 0, None, 60, queue_response=q)
        results = []
        for i in range(5):          # frames alternate over the lanes (own streams + workspaces)
            p.process_frame({"stream_id": "g", "frame_id": i}, {})
            info, out = q.get_nowait()
            assert info["state"] == 0
            results.append(out["topk"])
        src = p.get_element("SyntheticFrames")      # frames live in FIFO FramePool slots
        frames = [src.frame_pool.view(s, src._shape, torch.uint8) for s in range(src.frame_pool.capacity)]
        model = ResNet50(seed=0, device="cuda")
        for i, r in enumerate(results):
            got = r.wait()
            prob, idx = model(frames[i % len(frames)])
            torch.cuda.synchronize()
            assert torch.equal(got["top_index"], idx.cpu())
            assert torch.allclose(got["top_prob"], prob.cpu(), rtol=1e-4, atol=1e-6)
            assert r.latency is not None and r.latency > 0
        assert p.share["gpu_lanes"] == lanes


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


def _diamond(streams: bool, repeat=12, size=2048):
    M = "aiko_services_amd.elements.gpu.tensor_ops"

    def el(name, cls_in, cls_out, params):
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in cls_in],
                "output": [{"name": n, "type": "tensor"} for n in cls_out], "parameters": params,
                "deploy": {"local": {"module": M, "class_name": name.rstrip("AB")}}}
    pa = {"repeat": repeat, "seed": 1}
    pb = {"repeat": repeat, "seed": 2}
    if streams:
        pa["hip_stream"], pb["hip_stream"] = "branch_a", "branch_b"
    return {"version": 0, "name": "p_diamond", "runtime": "python",
            "graph": ["(GpuTensorSource (GpuMatChainA GpuAdd) (GpuMatChainB GpuAdd))"], "parameters": {},
            "elements": [el("GpuTensorSource", [], ["x"], {"size": size}),
                         el("GpuMatChainA", ["x"], ["ya"], pa),
                         el("GpuMatChainB", ["x"], ["yb"], pb),
                         el("GpuAdd", ["ya", "yb"], ["z"], {})]}


def test_branches_on_hip_streams_match_sequential(native):
    """Diamond graph: branches on two HIP streams (concurrent) give the sequential result."""
    import queue
    import time
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    results, times = {}, {}
    for streams in (False, True):
        q = queue.Queue()
        p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(_diamond(streams)), None, None,
                                         f"s{int(streams)}", [], 0, None, 60, queue_response=q)
        for i in range(3):          # warm-up
            p.process_frame({"stream_id": f"s{int(streams)}", "frame_id": i}, {})
            q.get(timeout=60)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(3, 13):
            p.process_frame({"stream_id": f"s{int(streams)}", "frame_id": i}, {})
            info, out = q.get(timeout=60)
            assert info["state"] == 0, out
        torch.cuda.synchronize()
        times[streams] = time.perf_counter() - t0
        results[streams] = out["z"].float().clone()
    assert torch.allclose(results[False], results[True], atol=1e-2)
    print(f"diamond sequential {times[False]*1e3:.1f} ms, two streams {times[True]*1e3:.1f} ms")


def test_face_detector_example_pipeline(native):
    """examples/face: FaceDetector (single-class YOLOv8 on the HIP kernels) + ImageOverlay."""
    import json
    from pathlib import Path
    import numpy as np
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    d = json.loads((Path(__file__).resolve().parents[1] /
                    "aiko_services_amd/examples/face/face_pipeline.json").read_text())
    d["graph"] = ["(FaceDetector ImageOverlay)"]            # frames fed directly below
    d["elements"] = d["elements"][1:]
    d["elements"][0]["parameters"] = {"conf": 0.01, "iou": 0.5, "image_size": 320}
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<face>", parse_pipeline_definition_dict(d), None, None, "f", [], 0,
                                     None, 60, queue_response=q)
    rng = np.random.default_rng(0)
    images = [rng.integers(0, 256, (240, 320, 3), dtype=np.uint8) for _ in range(3)]
    p.process_frame({"stream_id": "f", "frame_id": 0}, {"images": images})
    info, out = q.get(timeout=60)
    assert info["state"] == 0
    assert len(out["images"]) == 3 and out["images"][0].shape == (240, 320, 3)
    face = p.get_element("FaceDetector")
    assert face.model.nc == 1 and face.share["detections"] >= 0


def _run_bench_pipeline(d, frames):
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(d), None, None, "l", [], 0,
                                     None, 60, queue_response=q)
    outs = []
    for i in range(frames):
        p.process_frame({"stream_id": "l", "frame_id": i}, {})
        info, out = q.get_nowait()
        assert info["state"] == 0, out
        outs.append(next(iter(out.values())))
    return p, [{k: v.clone() for k, v in r.wait().items()} for r in outs]


@pytest.mark.parametrize("lanes", [2, 3])
def test_yolo_and_whisper_pipelines_lanes_match_single_lane(native, lanes):
    """Frame lanes change only the schedule: YOLOv8n detections and the Whisper sliding-window
    embeddings (a cross-frame state chained by events across lane streams) equal lanes=1."""
    import bench
    ref = _run_bench_pipeline(bench.yolo_definition(2, True, 240, 320, "scatter", 1), 5)[1]
    p, got = _run_bench_pipeline(bench.yolo_definition(2, True, 240, 320, "scatter", lanes), 5)
    assert p.share["gpu_lanes"] == lanes
    for a, b in zip(ref, got):
        assert torch.equal(a["count"], b["count"]) and torch.equal(a["det"], b["det"])
    ref = _run_bench_pipeline(bench.whisper_definition(2, True, "tiny", 2.0, 6.0, 1), 6)[1]
    p, got = _run_bench_pipeline(bench.whisper_definition(2, True, "tiny", 2.0, 6.0, lanes), 6)
    for a, b in zip(ref, got):
        assert torch.equal(a["pooled"], b["pooled"])


@pytest.mark.parametrize("chunk,blocks", [(32, 3), (16, 7)])
def test_resnet50_mall_chunking_matches(native, chunk, blocks):
    """Infinity-Cache blocking (stem + first bottlenecks per sub-batch) only reorders work:
    logits equal the whole-batch forward."""
    from aiko_services_amd.models.resnet50 import ResNet50
    g = torch.Generator().manual_seed(4)
    frames = torch.randint(0, 256, (64, 224, 224, 3), generator=g, dtype=torch.uint8).to("cuda")
    m = ResNet50(device="cuda")
    m.mall_chunk = 0
    ref = m.logits(frames).clone()
    m.mall_chunk, m.mall_blocks = chunk, blocks
    got = m.logits(frames).clone()
    assert torch.equal(got, ref) or ((got.float() - ref.float()).abs().max() < 1e-2 * ref.float().abs().max())


@pytest.mark.parametrize("k1,n1,n2", [(64, 256, 64), (64, 256, 128), (128, 512, 128)])
def test_conv_chain_matches_two_convs(native, k1, n1, n2, monkeypatch):
    """conv_chain (1x1 expand + residual + ReLU -> 1x1 reduce + ReLU in one kernel) equals the two
    separate igemm convs and the fp32 reference."""
    from aiko_services_amd.ops import conv as C
    g = torch.Generator().manual_seed(n2 + k1)
    spec3 = C.make_conv_spec(torch.randn(n1, k1, 1, 1, generator=g) / k1 ** 0.5, 0.1 * torch.randn(n1, generator=g),
                             act="relu", device="cuda")
    spec1 = C.make_conv_spec(torch.randn(n2, n1, 1, 1, generator=g) / n1 ** 0.5, 0.1 * torch.randn(n2, generator=g),
                             act="relu", device="cuda")
    assert C.chain_ok(spec3, spec1)
    B, H, W = 3, 28, 32                                      # M = 2688 = 42 tiles of 64
    x = torch.randn(B, H, W, k1, generator=g).to("cuda", torch.bfloat16)
    r = torch.randn(B, H, W, n1, generator=g).to("cuda", torch.bfloat16)
    y = torch.empty(B, H, W, n1, dtype=torch.bfloat16, device="cuda")
    z = torch.empty(B, H, W, n2, dtype=torch.bfloat16, device="cuda")
    for grid in (0, 5):                                      # persistent loop over several tiles
        C.conv_chain(x, spec3, r, y, spec1, z, grid=grid)
        y2 = C.conv2d(x, spec3, residual=r)
        z2 = C.conv2d(y2, spec1)
        assert ((y.float() - y2.float()).abs() > 0.02 * (1 + y2.float().abs())).float().mean() < 1e-3
        assert ((z.float() - z2.float()).abs().max() / z2.float().abs().max()) < 2e-2
        yr = torch.relu(x.float() @ spec3.ref_weight[:, :, 0, 0].T.cuda() + spec3.ref_bias.cuda() + r.float())
        assert ((y.float() - yr).norm() / yr.norm()).item() < 1e-2


def test_conv_chain_dual_matches_fused_conv(native):
    """Dual-source chain: [t2 | x] with the fused projection-shortcut weight (block 0 of stage 1)
    -> next block's reduction; equals conv2d(x2=...) followed by the 1x1 conv."""
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.models.resnet50 import ResNet50
    m = ResNet50(device="cuda")
    fused, nxt = m.blocks[0].fused, m.blocks[1].conv1
    assert C.chain_dual_ok(fused, nxt)
    g = torch.Generator().manual_seed(3)
    B, H, W = 2, 56, 56
    t2 = torch.randn(B, H, W, 64, generator=g).to("cuda", torch.bfloat16)
    x = torch.randn(B, H, W, 64, generator=g).to("cuda", torch.bfloat16)
    y = torch.empty(B, H, W, 256, dtype=torch.bfloat16, device="cuda")
    z = torch.empty(B, H, W, 64, dtype=torch.bfloat16, device="cuda")
    C.conv_chain(t2, fused, None, y, nxt, z, x2=x)
    y2 = C.conv2d(t2, fused, x2=x)
    z2 = C.conv2d(y2, nxt)
    assert ((y.float() - y2.float()).norm() / y2.float().norm()).item() < 5e-3
    assert ((z.float() - z2.float()).norm() / z2.float().norm()).item() < 1e-2


def test_resnet50_chain_matches_unchained(native):
    from aiko_services_amd.models.resnet50 import ResNet50
    g = torch.Generator().manual_seed(6)
    frames = torch.randint(0, 256, (16, 224, 224, 3), generator=g, dtype=torch.uint8).to("cuda")
    m = ResNet50(device="cuda")
    m.bneck = False              # stage 1 on the chained / patch kernels (bneck_fused replaces them)
    m.chain = False
    ref = m.logits(frames).float().clone()
    m.chain = True
    got = m.logits(frames).float()
    cos = torch.nn.functional.cosine_similarity(got.flatten(), ref.flatten(), dim=0).item()
    assert cos > 0.999, cos


def test_phase_gated_lanes_match_ungated(native):
    """Lane phase gating (two-part forward, stage 1-2 half waits for the previous frame's)
    gives bit-identical results to the single-graph forward."""
    import bench
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    outs = []
    for gate in (False, True):
        d = bench.definition(8, True, 224, 224, 2)
        d["elements"][1]["parameters"]["phase_gate"] = gate
        q = queue.Queue()
        p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(d), None, None, "g", [], 0, None, 60,
                                         queue_response=q)
        res = []
        for i in range(6):
            p.process_frame({"stream_id": "g", "frame_id": i}, {})
            res.append(q.get_nowait()[1]["topk"])
        outs.append([r.wait()["top_index"].clone() for r in res])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_run_maybe_captured_admission(native):
    """Per-address hipGraphs only for addresses that recur or are known stable (FramePool slots,
    static outputs of captured graphs): transient buffers run the copy-in graph and never pay a
    capture; per-address graphs are kept LRU."""
    from aiko_services_amd.gpu.element import FramePool, GpuPipelineElement

    class _El:                      # the graph-cache state of an element, without a pipeline
        use_graph, lane = True, 0
        max_graphs_per_key = GpuPipelineElement.max_graphs_per_key
        max_seen_addresses = GpuPipelineElement.max_seen_addresses
        run_maybe_captured = GpuPipelineElement.run_maybe_captured
        _retire_graph = GpuPipelineElement._retire_graph
    el = _El()
    el._captured = {}
    el.max_graphs_per_key = 2

    def fn(x):
        return x * 2 + 1
    keep = [torch.full((256,), float(i), device="cuda") for i in range(2)]
    for x in keep:                                      # warm phase: graphs at first sight
        assert torch.equal(el.run_maybe_captured("k", fn, x), x * 2 + 1)
    graphs = el._captured[("graphs", "k", 0)]
    assert len(graphs) == 2
    transient = [torch.full((256,), 10.0 + i, device="cuda") for i in range(4)]   # distinct addresses
    for x in transient:                                 # cache full: transient inputs, no capture
        assert torch.equal(el.run_maybe_captured("k", fn, x), x * 2 + 1)
    assert list(graphs) == [(t.data_ptr(),) for t in keep]
    x = torch.zeros(256, device="cuda")                 # a recurring address: graph on 2nd visit
    for v in (3.0, 4.0, 5.0):
        x.fill_(v)
        assert torch.equal(el.run_maybe_captured("k", fn, x), x * 2 + 1)
    assert list(graphs) == [(keep[1].data_ptr(),), (x.data_ptr(),)]     # LRU dropped the oldest
    pool = FramePool(2, 1024, device="cuda:0")         # a pool slot: captured at first sight
    slot = pool.view(pool.acquire(0.1), (256,), torch.float32)
    slot.fill_(7.0)
    assert torch.equal(el.run_maybe_captured("k", fn, slot), slot * 2 + 1)
    assert list(graphs) == [(x.data_ptr(),), (slot.data_ptr(),)]
    slot.fill_(-1.0)
    assert torch.equal(el.run_maybe_captured("k", fn, slot), slot * 2 + 1)
    torch.cuda.synchronize()
