"""Pipeline parallelism (BASELINE config 3 topology) on CPU: one process per stage, gloo P2P.

The same StageLink / PipelineParallelRunner code runs over RCCL on MI355X; here world sizes 2
and 3 check stage splitting, signature exchange, slot rings with look-ahead receives, header
propagation (frame id, DROP_FRAME state, submit stamp) and the end-of-stream terminator.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from aiko_services_amd.parallel.pipeline_parallel import split_stages, element_chain
from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict

MOD = "aiko_services_amd.elements.tensor"


def _definition(stages=None, drop_every=0, batch=2, size=8):
    def el(name, cls_in, cls_out, params=None, stage=None):
        local = {"module": MOD}
        if stage is not None:
            local["stage"] = stage
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in cls_in],
                "output": [{"name": n, "type": "tensor"} for n in cls_out],
                "parameters": params or {}, "deploy": {"local": local}}
    s = stages or [None] * 4
    return {
        "version": 0, "name": "p_pp_test", "runtime": "python",
        "graph": ["(TensorSource TensorDrop TensorAffine TensorReduce)"], "parameters": {},
        "elements": [
            el("TensorSource", [], ["x"], {"batch": batch, "size": size}, s[0]),
            el("TensorDrop", ["x"], ["x"], {"every": drop_every}, s[1]),
            el("TensorAffine", ["x"], ["x"], {"scale": 2.0, "offset": 1.0}, s[2]),
            el("TensorReduce", ["x"], ["y"], {}, s[3]),
        ],
    }


def test_split_stages():
    d = parse_pipeline_definition_dict(_definition())
    assert element_chain(d) == ["TensorSource", "TensorDrop", "TensorAffine", "TensorReduce"]
    assert split_stages(d, 2) == [["TensorSource", "TensorDrop"], ["TensorAffine", "TensorReduce"]]
    assert split_stages(d, 3) == [["TensorSource", "TensorDrop"], ["TensorAffine"], ["TensorReduce"]]
    d = parse_pipeline_definition_dict(_definition(stages=[0, 0, 0, 1]))
    assert split_stages(d, 2) == [["TensorSource", "TensorDrop", "TensorAffine"], ["TensorReduce"]]
    with pytest.raises(ValueError):
        split_stages(parse_pipeline_definition_dict(_definition(stages=[1, 0, 1, 1])), 2)
    with pytest.raises(ValueError):
        split_stages(parse_pipeline_definition_dict(_definition()), 5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, drop_every, results):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "AIKO_MQTT_DISABLE": "1", "AIKO_LOG_MQTT": "false", "AIKO_LOG_LEVEL": "WARNING"})
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel.pipeline_parallel import PipelineParallelRunner
    D.init("gloo")
    try:
        d = parse_pipeline_definition_dict(_definition(drop_every=drop_every))
        runner = PipelineParallelRunner(d, device="cpu", depth=2)
        out = []
        for _ in range(frames):
            r = runner.step({})
            if r is not None:
                info, data = r
                out.append((int(info["header"][0]), PipelineParallelRunner.upstream_state(info),
                            data["y"].tolist(), int(info["header"][2]) > 0))
        runner.finish()
        if runner.is_last:
            results.put(out)
        D.barrier()
    finally:
        D.destroy()


@pytest.mark.parametrize("world,drop_every", [(2, 0), (3, 3)])
def test_pipeline_parallel_gloo(world, drop_every):
    frames, size = 7, 8
    ctx = mp.get_context("spawn")
    results = ctx.SimpleQueue()
    mp.spawn(_worker, args=(world, _free_port(), frames, drop_every, results), nprocs=world, join=True)
    out = results.get()
    assert [o[0] for o in out] == list(range(frames))
    for fid, state, y, stamped in out:
        expect = sum((k + fid) * 2.0 + 1.0 for k in range(size))
        assert y == [expect, expect]
        assert stamped
        dropped = drop_every and fid % drop_every == drop_every - 1
        assert state == (1 if dropped else 0), (fid, state)


def _fault_worker(rank, world, port, results):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "AIKO_MQTT_DISABLE": "1", "AIKO_LOG_MQTT": "false", "AIKO_LOG_LEVEL": "ERROR"})
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel.pipeline_parallel import PipelineParallelRunner, StageFailure
    from aiko_services_amd.utils import fault
    D.init("gloo", timeout_s=30)
    if rank == 1:
        fault.inject("kill=3")            # the middle stage dies after its 3rd frame
    d = parse_pipeline_definition_dict(_definition(batch=64, size=64))
    runner = PipelineParallelRunner(d, device="cpu", depth=2)
    ok = 0
    try:
        for _ in range(200):
            runner.step({})
            ok += 1
        results.put((rank, "no failure", ok))
    except StageFailure as exc:
        share = runner.pipeline.share
        results.put((rank, exc.peer, ok, share["lifecycle"], share.get("stage_failed")))
    os._exit(0)                          # the group is broken: skip the collective teardown


def test_stage_rank_failure_detected():
    """Fault injection (kill a stage rank): both neighbours observe StageFailure naming it."""
    world = 3
    ctx = mp.get_context("spawn")
    results = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_fault_worker, args=(r, world, port, results)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    from aiko_services_amd.utils.fault import KILL_EXIT_CODE
    assert procs[1].exitcode == KILL_EXIT_CODE
    got = {}
    while not results.empty():
        r = results.get()
        got[r[0]] = r[1:]
    assert got[0][0] == 1 and got[0][2:] == ("waiting", 1), got
    assert got[2][0] == 1 and got[2][2:] == ("waiting", 1), got
    assert got[2][1] <= 3
