"""Data-plane bootstrap over the MQTT control plane (in-repo broker) + the hop data plane, on
CPU with gloo (the same path initialises RCCL on MI355X)."""
import os

import torch
import torch.multiprocessing as mp

from aiko_services_amd.message.mqtt_broker import start_broker_thread


def _worker(rank, world, port, ns, results, mailboxes):
    os.environ.update({"AIKO_NAMESPACE": ns, "AIKO_MQTT_DISABLE": "1", "AIKO_LOG_LEVEL": "WARNING",
                       "AIKO_RENDEZVOUS_HOST": "127.0.0.1"})
    import torch.distributed as tdist
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel.hop import HopPlane
    from aiko_services_amd.parallel.rendezvous import rendezvous_init
    assert rendezvous_init("testgroup", rank, world, "127.0.0.1", port, backend="gloo", timeout_s=30)
    t = torch.tensor([float(rank + 1)])
    tdist.all_reduce(t)
    # a 3-rank chain over the hop plane: 0 -> 1 -> 2 (token dicts stand in for the MQTT
    # process_frame metadata; the tensors travel on the per-direction gloo/RCCL links)
    from aiko_services_amd.parallel.hop import mark_frame_held
    plane = HopPlane([(0, 1), (1, 2)], device="cpu", depth=2)
    out = None
    if rank == 0:
        for i in range(3):
            mailboxes[1].put(plane.encode(1, {"x": torch.full((4,), float(i)), "i": i}))
        # a frame-held tensor alone in a forward hop: sent from its own storage (no staging)
        held = mark_frame_held(torch.arange(6, dtype=torch.int32).reshape(2, 3))
        mailboxes[1].put(plane.encode(1, {"y": held}, key=("s", 9)))
        out = (plane.counters["zero_copy"], plane.credit(1))
        mailboxes[0].get()                        # rank 1 decoded it: acknowledge (credit back)
        plane.ack(("s", 9))
        out = out + (plane.credit(1),)
    elif rank == 1:
        for _ in range(3):
            vals, handle = plane.decode(mailboxes[1].get())
            mailboxes[2].put(plane.encode(2, {"x": vals["x"] * 10, "i": vals["i"]}))
            plane.release([handle])
        vals, handle = plane.decode(mailboxes[1].get())
        out = vals["y"].tolist()
        plane.release([handle])
        mailboxes[0].put("ok")
    else:
        got = []
        for _ in range(3):
            vals, handle = plane.decode(mailboxes[2].get())
            got.append((int(vals["i"]), vals["x"].tolist()))
            plane.release([handle])
        out = got
    plane.close()
    results.put((rank, float(t.item()), out))
    D.barrier()
    D.destroy()


def test_mqtt_rendezvous_and_hop_chain():
    broker, port = start_broker_thread("127.0.0.1", 0)
    try:
        world = 3
        ctx = mp.get_context("spawn")
        results = ctx.SimpleQueue()
        mailboxes = [ctx.SimpleQueue() for _ in range(world)]
        mp.spawn(_worker, args=(world, port, "rdvtest", results, mailboxes), nprocs=world, join=True)
        got = {r: (s, o) for r, s, o in (results.get() for _ in range(world))}
        assert all(s == 6.0 for s, _ in got.values())
        assert got[2][1] == [(i, [10.0 * i] * 4) for i in range(3)]
        assert got[1][1] == [[0, 1, 2], [3, 4, 5]]
        assert got[0][1] == (1, 1, 2)                 # one zero-copy send; its credit held, then back
    finally:
        broker.stop()
