"""Data-parallel fan-out / gather (BASELINE config 4 topology) on CPU with gloo.

The ingest rank produces the node's whole frame batch, FrameFanout hands each rank its slice
(scatter = grouped P2P, broadcast = whole batch + local slice), a stand-in detector emits
fixed-size rows, DetectionsGather all-gathers them; every rank must end up with the
detections of the whole batch in rank order.  The same elements run over RCCL on MI355X.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

B, H, W = 3, 8, 12
SEED = 7


def _definition(mode):
    def el(name, module, inputs, outputs, params):
        params = dict(params, device="cpu")
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in inputs],
                "output": [{"name": n, "type": "tensor"} for n in outputs],
                "parameters": params, "deploy": {"local": {"module": module}}}
    return {
        "version": 0, "name": "p_dp_test", "runtime": "python",
        "graph": ["(SyntheticFrames FrameFanout FrameStats DetectionsGather)"], "parameters": {},
        "elements": [
            el("SyntheticFrames", "aiko_services_amd.elements.gpu.vision", [], ["images", "t_submit"],
               {"batch": B, "height": H, "width": W, "pool": 2, "global": True, "seed": SEED}),
            el("FrameFanout", "aiko_services_amd.elements.gpu.detect", ["images"], ["images"],
               {"mode": mode, "batch": B, "height": H, "width": W}),
            el("FrameStats", "aiko_services_amd.elements.tensor", ["images"], ["detections", "counts"], {}),
            el("DetectionsGather", "aiko_services_amd.elements.gpu.detect",
               ["detections", "counts", "t_submit"], ["detections"], {}),
        ],
    }


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, mode, frames, results):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "AIKO_MQTT_DISABLE": "1", "AIKO_LOG_MQTT": "false", "AIKO_LOG_LEVEL": "WARNING"})
    import queue
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    D.init("gloo")
    try:
        q = queue.Queue()
        p = PipelineImpl.create_pipeline("<dp>", parse_pipeline_definition_dict(_definition(mode)), None,
                                         None, "dp", [], 0, None, 3600, queue_response=q)
        out = []
        for i in range(frames):
            p.process_frame({"stream_id": "dp", "frame_id": i}, {})
            info, data = q.get_nowait()
            assert info["state"] == 0, data
            r = data["detections"].wait()
            out.append((r["det"].tolist(), r["count"].tolist()))   # plain data: workers exit first
        results.put((rank, (out, D.comm_stats())))
        D.barrier()
    finally:
        D.destroy()


@pytest.mark.parametrize("mode,world", [("scatter", 2), ("broadcast", 3)])
def test_dp_fanout_gather(mode, world):
    frames = 3
    ctx = mp.get_context("spawn")
    results = ctx.SimpleQueue()
    mp.spawn(_worker, args=(world, _free_port(), mode, frames, results), nprocs=world, join=True)
    got = dict(results.get() for _ in range(world))
    stats = {r: v[1] for r, v in got.items()}
    got = {r: v[0] for r, v in got.items()}
    frame_bytes = B * H * W * 3
    for r, st in stats.items():   # RCCL byte counters: exact per-rank accounting
        assert st["all_gather"]["calls"] >= frames
        if mode == "broadcast":
            assert st["broadcast"] == {"calls": frames, "bytes": frames * world * frame_bytes}
        elif r == 0:
            assert st["send"] == {"calls": frames * (world - 1), "bytes": frames * (world - 1) * frame_bytes}
        else:
            assert st["recv"] == {"calls": frames, "bytes": frames * frame_bytes}
    g = torch.Generator(device="cpu").manual_seed(SEED)
    pool = [torch.randint(0, 256, (world * B, H, W, 3), dtype=torch.uint8, generator=g) for _ in range(2)]
    for i in range(frames):
        f = pool[i % 2].float()
        expect = torch.cat([f.mean(dim=(1, 2)), f.mean(dim=(1, 2, 3))[:, None]], 1)
        for rank in range(world):
            det, count = torch.tensor(got[rank][i][0]), torch.tensor(got[rank][i][1])
            assert det.shape == (world * B, 1, 6)
            assert torch.allclose(det[:, 0, :4], expect, atol=1e-4), (rank, i)
            assert (count == 1).all()
