"""RCCL code paths on ONE MI355X (launched by tests/test_gpu_rccl.py under
``torch.distributed.run --nproc-per-node 1``): process-group init on the ``nccl`` backend with
``device_id``, ``barrier(device_ids=...)``, all-gathers issued from both frame-lane streams in
the engine's order, ClassifierTopK's gather, and the hop data plane (loopback link: staging
ring, FramePool receive slot, event-gated release, DeviceResult rebuild) on device tensors."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from aiko_services_amd.gpu.element import DeviceResult  # noqa: E402
from aiko_services_amd.gpu.lanes import lane_scope  # noqa: E402
from aiko_services_amd.parallel import dist as D  # noqa: E402
from aiko_services_amd.parallel import hop  # noqa: E402


def main():
    assert D.init(backend_name="nccl", force=True), "process group not created"
    assert D.backend() == "nccl" and D.world_size() == 1
    dev = torch.device("cuda", torch.cuda.current_device())
    D.barrier()
    # all-gathers from the two lane streams, interleaved the way frame lanes issue them
    outs = []
    for k in range(4):
        with lane_scope(k % 2, dev):
            t = torch.full((8, 5), float(k), device=dev)
            o = torch.empty(8, 5, device=dev)
            D.all_gather_into(o, t)
            outs.append(o)
    torch.cuda.synchronize()
    for k, o in enumerate(outs):
        assert torch.equal(o, torch.full((8, 5), float(k), device=dev)), k
    # hop plane over a loopback link: tensors + a DeviceResult + a float
    plane = hop.init_plane([(0, 0)], device=dev, depth=2)
    for k in range(6):
        x = torch.randn(3, 224, 224, device=dev).to(torch.bfloat16)
        idx = torch.arange(7, dtype=torch.int32, device=dev) + k
        hp = torch.randn(4, 5).pin_memory()
        ev = torch.cuda.Event()
        ev.record()
        msg = plane.encode(0, {"x": x, "n": 3, "t": 1.5 + k, "r": DeviceResult({"p": hp, "i": idx}, ev, t_submit=2.5)})
        assert isinstance(msg["x"], str) and msg["x"].startswith("T@0/"), msg
        got, handle = plane.decode(msg, pooled=True)
        assert handle is not None, "forward hop must land in a FramePool slot"
        assert torch.equal(got["x"], x) and got["n"] == 3 and got["t"] == 1.5 + k
        r = got["r"]
        assert isinstance(r, DeviceResult) and r.t_submit == 2.5
        res = r.wait()
        assert torch.equal(res["p"].cpu(), hp) and torch.equal(res["i"], idx)
        plane.release([handle])
    torch.cuda.synchronize()
    st = plane.stats()
    assert st["pool_overflow"] == 0 and st["recv_msgs"] == 6, st
    hop.shutdown_plane()
    D.barrier()
    D.destroy()
    print("RCCL_WORLD1_OK", flush=True)


if __name__ == "__main__":
    main()
