"""Data-plane bootstrap over the MQTT control plane (in-repo broker) + TensorChannels, on CPU
with gloo (the same path initialises RCCL on MI355X)."""
import os

import torch
import torch.multiprocessing as mp

from aiko_services_amd.message.mqtt_broker import start_broker_thread
from aiko_services_amd.message.tensor_channel import LoopbackTensorChannel


def _worker(rank, world, port, ns, results):
    os.environ.update({"AIKO_NAMESPACE": ns, "AIKO_MQTT_DISABLE": "1", "AIKO_LOG_LEVEL": "WARNING",
                       "AIKO_RENDEZVOUS_HOST": "127.0.0.1"})
    import torch.distributed as tdist
    from aiko_services_amd.message.tensor_channel import RcclTensorChannel
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel.rendezvous import rendezvous_init
    assert rendezvous_init("testgroup", rank, world, "127.0.0.1", port, backend="gloo", timeout_s=30)
    t = torch.tensor([float(rank + 1)])
    tdist.all_reduce(t)
    # a 3-rank chain over TensorChannels: 0 -> 1 -> 2
    out = None
    if rank == 0:
        ch = RcclTensorChannel(1, "send", device="cpu")
        for i in range(3):
            ch.send([i, 0, 0, 0], {"x": torch.full((4,), float(i))})
        ch.close()
    elif rank == 1:
        rx, tx = RcclTensorChannel(0, "recv", device="cpu"), RcclTensorChannel(2, "send", device="cpu")
        for _ in range(3):
            hdr, t_ = rx.recv()
            tx.send(hdr, {"x": t_["x"] * 10})
        tx.close()
    else:
        rx = RcclTensorChannel(1, "recv", device="cpu")
        got = []
        for _ in range(3):
            hdr, t_ = rx.recv()
            got.append((hdr[0], t_["x"].tolist()))
        out = got
    results.put((rank, float(t.item()), out))
    D.barrier()
    D.destroy()


def test_mqtt_rendezvous_and_rccl_channels():
    broker, port = start_broker_thread("127.0.0.1", 0)
    try:
        world = 3
        ctx = mp.get_context("spawn")
        results = ctx.SimpleQueue()
        mp.spawn(_worker, args=(world, port, "rdvtest", results), nprocs=world, join=True)
        got = {r: (s, o) for r, s, o in (results.get() for _ in range(world))}
        assert all(s == 6.0 for s, _ in got.values())
        assert got[2][1] == [(i, [10.0 * i] * 4) for i in range(3)]
    finally:
        broker.stop()


def test_loopback_channel_zero_copy():
    ch = LoopbackTensorChannel()
    x = torch.arange(4)
    ch.send([7, 0], {"x": x})
    hdr, t = ch.recv(timeout=1)
    assert hdr == [7, 0] and t["x"] is x
