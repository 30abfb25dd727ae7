"""FrameUpload (host -> HBM ingest): uploaded frame batches are bit-equal to
the host frames — pinned batches from SyntheticFrames(host), pageable tensors and lists of
numpy images (VideoReadFile / ImageReadFile / webcam outputs) — and kernels that the frame's
stream runs right after the upload see the uploaded bytes (the copy runs on the element's
own copy stream; the frame's stream waits on its event)."""
import queue

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pipeline(batch=8, h=96, w=128, pool=3):
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    mod = "aiko_services_amd.elements.gpu.vision"
    d = {"version": 0, "name": "p_upload", "runtime": "python", "graph": ["(SyntheticFrames FrameUpload)"],
         "parameters": {},
         "elements": [
             {"name": "SyntheticFrames", "input": [], "output": [{"name": "images", "type": "tensor"},
                                                                {"name": "t_submit", "type": "float"}],
              "parameters": {"batch": batch, "height": h, "width": w, "pool": pool, "host": True, "seed": 5},
              "deploy": {"local": {"module": mod}}},
             {"name": "FrameUpload", "input": [{"name": "images", "type": "tensor"}],
              "output": [{"name": "images", "type": "tensor"}], "parameters": {"pool": 4},
              "deploy": {"local": {"module": mod}}}]}
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<upload>", parse_pipeline_definition_dict(d), None, None, "up", [], 0,
                                     None, 60, queue_response=q)
    return p, q


def test_upload_pipeline_frames_bit_equal(native):
    p, q = _pipeline()
    src = p.pipeline_graph.get_node("SyntheticFrames").element
    sums = []
    for fid in range(7):
        p.process_frame({"stream_id": "up", "frame_id": fid}, {})
        info, out = q.get_nowait()
        assert info["state"] == 0, out
        img = out["images"]
        assert img.is_cuda and img.dtype == torch.uint8 and tuple(img.shape) == (8, 96, 128, 3)
        # a kernel on the current stream right after the upload (no synchronize in between)
        sums.append(img.to(torch.int64).sum())
        host = src.host_pool[fid % 3]
        assert torch.equal(img.cpu(), host), fid
    expect = [int(src.host_pool[f % 3].to(torch.int64).sum()) for f in range(7)]
    assert [int(s) for s in sums] == expect


def test_upload_pageable_and_numpy_lists(native):
    p, _ = _pipeline()
    up = p.pipeline_graph.get_node("FrameUpload").element
    g = torch.Generator().manual_seed(3)
    batch = torch.randint(0, 256, (5, 40, 60, 3), dtype=torch.uint8, generator=g)     # pageable
    ev, out = up.process_frame(None, images=batch)
    assert ev == 0 and torch.equal(out["images"].cpu(), batch)
    imgs = [np.random.default_rng(i).integers(0, 256, (40, 60, 3), dtype=np.uint8) for i in range(5)]
    outs = []
    for k in range(6):                        # more uploads than staging sets: ring reuse
        ev, out = up.process_frame(None, images=imgs)
        outs.append(out["images"].clone())
    torch.cuda.synchronize()
    want = torch.from_numpy(np.stack(imgs))
    assert all(torch.equal(o.cpu(), want) for o in outs)
    ev, out = up.process_frame(None, images=imgs[0])                      # one HxWx3 image
    assert torch.equal(out["images"].cpu()[0], torch.from_numpy(imgs[0]))
