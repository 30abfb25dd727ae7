"""Multi-GPU actor pipelines on the CPU (gloo): ``aiko_pipeline create`` of a definition with
``parallel: {mode: pp, gpus: 3}`` spawns one registered worker Pipeline per stage, tensors
cross the stage boundaries over the hop data plane (``parallel/hop.py``) while MQTT carries
only metadata, and the outputs match the single-process run bit for bit."""
import json
import os
import re
import subprocess
import sys
import tempfile
import time
import uuid

import pytest

from aiko_services_amd.message.mqtt_broker import start_broker_thread

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFS = os.path.join(ROOT, "aiko_services_amd", "examples", "pipeline", "definitions")


@pytest.fixture
def cluster():
    broker, port = start_broker_thread("127.0.0.1", 0)
    payloads = []
    broker.on_publish = lambda topic, payload: payloads.append((topic, bytes(payload)))
    env = dict(os.environ)
    env.update({"AIKO_MQTT_HOST": "127.0.0.1", "AIKO_MQTT_PORT": str(port),
                "AIKO_NAMESPACE": f"t{uuid.uuid4().hex[:8]}", "AIKO_LOG_MQTT": "false",
                "AIKO_LOG_LEVEL": "WARNING", "AIKO_REGISTRAR_SEARCH_TIMEOUT": "0.3",
                "AIKO_MQTT_DISABLE": "0", "AIKO_HOP_BACKEND": "gloo", "OMP_NUM_THREADS": "1",
                "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
    procs = []
    reg = subprocess.Popen([sys.executable, "-m", "aiko_services_amd.tools.registrar"], env=env, cwd=ROOT,
                           stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    procs.append(reg)
    time.sleep(0.8)
    yield {"env": env, "payloads": payloads, "broker": broker}
    for p in procs:
        p.terminate()
        try:
            p.wait(5)
        except subprocess.TimeoutExpired:
            p.kill()
    broker.stop()


def _outputs(text):
    return {int(m.group(1)): m.group(2) for m in re.finditer(r"Output: <1:(\d+)> (.*)", text)}


def _create(env, path, frames, timeout=120):
    r = subprocess.run([sys.executable, "-m", "aiko_services_amd.pipeline.cli", "create", path,
                        "-s", "1", "-x", str(frames), "-sr", "-ll", "INFO", "-lm", "false"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    return r, _outputs(r.stdout + r.stderr)


def test_pp3_actor_pipeline_matches_single_process(cluster):
    path = os.path.join(DEFS, "tensor_pp3.json")
    r, par = _create(cluster["env"], path, 6)
    assert len(par) == 6, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    assert all("sha=" in v for v in par.values()), par
    # the metadata plane carried tensor tokens, never tensor bytes
    hops = [p for t, p in cluster["payloads"] if b"process_frame" in p]
    assert any(b"T@" in p for p in hops), "no tensor tokens seen on MQTT"
    assert max(len(p) for _, p in cluster["payloads"]) < 4096
    # same definition in ONE process (no parallel block, no stages)
    with open(path) as f:
        d = json.load(f)
    d.pop("parallel")
    for e in d["elements"]:
        e["deploy"]["local"].pop("stage")
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(d, f)
    try:
        r1, single = _create(cluster["env"], f.name, 6)
    finally:
        os.unlink(f.name)
    assert single == par, (single, par)


def test_plan_nested_stages():
    from aiko_services_amd.parallel.placement import make_plan
    with open(os.path.join(DEFS, "tensor_pp3.json")) as f:
        d = json.load(f)
    plan = make_plan(d)
    assert plan.world == 3 and plan.stages == [["TensorFrames"], ["TensorAffine"], ["TensorStats"]]
    assert plan.ranks[0].definition["graph"] == ["(TensorFrames Stage1)"]
    assert plan.ranks[1].definition["graph"] == ["(TensorAffine Stage2)"]
    assert plan.ranks[2].definition["graph"] == ["(TensorStats)"]
    remote = plan.ranks[1].definition["elements"][-1]
    assert remote["deploy"]["remote"]["service_filter"]["name"] == "p_tensor_pp_s2"
    assert [i["name"] for i in remote["input"]] == ["t_submit", "x"]
    assert sorted(map(tuple, plan.links)) == [(0, 1), (1, 0), (1, 2), (2, 1)]


def test_replicated_stage_matches_single_process(cluster):
    """Stage 1 replicated on ranks 1 and 2 plus an in-process copy on rank 0 (PP x DP)."""
    path = os.path.join(DEFS, "tensor_ppdp.json")
    r, par = _create(cluster["env"], path, 8)
    assert len(par) == 8, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    sent = {}
    for topic, p in cluster["payloads"]:
        if p.startswith(b"(process_frame ") and b"T@0/" in p:
            sent[topic] = sent.get(topic, 0) + 1
    assert len(sent) == 2, sent                       # both remote replicas got frames
    with open(path) as f:
        d = json.load(f)
    d.pop("parallel")
    for e in d["elements"]:
        e["deploy"]["local"].pop("stage")
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump(d, f)
    try:
        _, single = _create(cluster["env"], f.name, 8)
    finally:
        os.unlink(f.name)
    assert single == par


def test_balancer_replicates_the_heavy_stage():
    """Config 3 element times (1-GPU profile, ms per 256-frame batch): the planner replicates
    ResNet-50 and gives rank 0 a share of it, so per-rank times are within 15 %."""
    from aiko_services_amd.parallel.placement import plan_stages
    order = ["SyntheticFrames", "ImagePreprocess", "ResNet50Classifier", "ClassifierTopK"]
    times = {"SyntheticFrames": 0.01, "ImagePreprocess": 0.12, "ResNet50Classifier": 3.35,
             "ClassifierTopK": 0.03}
    for gpus in (2, 4, 8):
        stages, reps, share, per_rank = plan_stages(order, times, gpus)
        assert len(per_rank) == gpus, (stages, reps, share)
        assert max(per_rank) <= 1.15 * min(per_rank), (gpus, stages, reps, share, per_rank)
        assert max(per_rank) < sum(times.values()) / gpus * 1.1


def test_hop_loopback_cpu():
    """Hop encode/decode on a loopback link (no process group): tokens, packing, FramePool
    slot, float and DeviceResult round trip."""
    import torch
    from aiko_services_amd.gpu.element import DeviceResult
    from aiko_services_amd.parallel.hop import HopPlane
    plane = HopPlane([(0, 0)], device="cpu", depth=2)
    x = torch.randn(5, 7)
    msg = plane.encode(0, {"x": x, "s": "keep", "t": 0.25,
                           "r": DeviceResult({"a": torch.arange(3)}, None, t_submit=1.0)})
    assert msg["s"] == "keep" and msg["t"] == "F@0.25" and msg["x"].startswith("T@0/0/0/float32/5x7")
    got, handle = plane.decode(msg)
    assert torch.equal(got["x"], x) and got["t"] == 0.25 and got["s"] == "keep"
    assert torch.equal(got["r"].wait()["a"], torch.arange(3)) and got["r"].t_submit == 1.0
    plane.release([handle])
    handle[0].acquire(0.0)                  # retires the pending release (CPU: immediate)
    assert plane.stats()["pool_free_from_0"] == 3


def test_dp_spmd_actor_pipeline(cluster):
    """``parallel: {mode: dp, gpus: 2}`` through ``aiko_pipeline create``: both ranks run the
    whole pipeline on the same stream; rank 0's results hold the all-gathered rows of both."""
    r, out = _create(cluster["env"], os.path.join(DEFS, "tensor_dp2.json"), 4)
    assert len(out) == 4, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    for v in out.values():
        assert "float32,6x1x6" in v and "int32,6" in v, v      # world x batch rows gathered
