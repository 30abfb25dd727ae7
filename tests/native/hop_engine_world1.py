"""Engine-level remote-hop path at world 1 on ONE GPU: two stage Pipelines
in one process joined over the hop plane's loopback link (hop_rank 0), an in-process message
bus, ``gpu_lanes`` 2 on both, ``hop_batch`` 4 and link depth 2 — so frames queue for credits and
the engine's own ``_queue_hop`` -> ``_drain_pending`` -> ``_dispatch_group`` -> (stage 1)
``_process_group`` -> ``_flush_responses`` path carries device tensors produced on one lane and
sent from another (the producer sleeps on the GPU before writing them).  Prints ``RESULT
{json}``: the per-frame outputs of the 2-stage run and of the single-stage pipeline.

    python tests/native/hop_engine_world1.py [--no-order]   # --no-order: _order_after stubbed
Reference: the remote PipelineElement hand-off, /root/reference/src/aiko_services/main/pipeline.py:1072-1103."""
import hashlib
import json
import os
import queue
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ["AIKO_MQTT_DISABLE"] = "1"
os.environ.setdefault("AIKO_LOG_LEVEL", "WARNING")
os.environ.setdefault("AIKO_LOG_MQTT", "false")

import torch  # noqa: E402

FRAMES = 24
MOD = "aiko_services_amd.examples.pipeline.tensor_elements"


def el(name, inputs, outputs, params=None):
    return {"name": name, "input": [{"name": n, "type": "tensor"} for n in inputs],
            "output": [{"name": n, "type": "tensor"} for n in outputs], "parameters": params or {},
            "deploy": {"local": {"module": MOD}}}


def definitions(device="cuda:0"):
    params = {"device": device, "batch": 64, "width": 4096, "gpu_lanes": 2, "hop_batch": 4}
    frames = el("TensorFrames", [], ["x", "t_submit"], {"frames": FRAMES, "gpu_sleep": 20_000_000})
    affine = el("TensorAffine", ["x"], ["x"], {"scale": "3.0", "shift": "-0.25"})
    stats = el("TensorStats", ["x", "t_submit"], ["stats"])
    single = {"version": 0, "name": "p_w1_single", "runtime": "python", "parameters": dict(params),
              "graph": ["(TensorFrames TensorAffine TensorStats)"], "elements": [frames, affine, stats]}
    s1 = {"version": 0, "name": "p_w1_s1", "runtime": "python", "parameters": dict(params),
          "graph": ["(TensorAffine TensorStats)"], "elements": [affine, stats]}
    remote = {"name": "Stage1", "input": [{"name": "x", "type": "tensor"}, {"name": "t_submit", "type": "float"}],
              "output": [{"name": "stats", "type": "result"}],
              "deploy": {"remote": {"module": "aiko_services_amd.pipeline.engine",
                                    "service_filter": {"name": "p_w1_s1"}}}}
    s0 = {"version": 0, "name": "p_w1_s0", "runtime": "python", "parameters": dict(params),
          "graph": ["(TensorFrames Stage1)"], "elements": [frames, remote]}
    return single, s0, s1


def digest(out):
    res = out["stats"].wait() if hasattr(out["stats"], "wait") else out["stats"]
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    h = hashlib.sha256()
    for k in ("sum", "max"):
        h.update(res[k].detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()[:16]


def run_stream(pipeline, sid, q):
    from aiko_services_amd.runtime.actor import ActorTopic
    pipeline._post_message(ActorTopic.IN, "create_stream", [sid, None, {}, 600, q, None])
    outs = {}
    deadline = time.time() + 120
    while len(outs) < FRAMES and time.time() < deadline:
        try:
            info, out = q.get(timeout=1.0)
        except queue.Empty:
            continue
        if info.get("state", 0) != 0:
            raise RuntimeError(f"frame failed: {info} {out}")
        outs[int(info["frame_id"])] = digest(out)
    return outs


def main():
    from aiko_services_amd.message.message import Loopback
    from aiko_services_amd.parallel import hop
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    from aiko_services_amd.runtime.process import aiko
    if "--no-order" in sys.argv:          # negative control: the pre-round-4 behaviour
        hop.HopPlane._order_after = lambda self, events: None
    cpu = "--cpu" in sys.argv              # (debugging the plumbing without a GPU: one lane)
    dev = torch.device("cpu") if cpu else torch.device("cuda", 0)
    if not cpu:
        torch.cuda.set_device(0)
    aiko.process.run_in_thread(message=Loopback())
    plane = hop.init_plane([(0, 0)], device=dev, depth=2)
    single_d, s0_d, s1_d = definitions("cpu" if cpu else "cuda:0")

    def create(d, name):
        return PipelineImpl.create_pipeline(f"<{name}>", parse_pipeline_definition_dict(d), name, None,
                                            None, [], 0, None, 600)

    single = create(single_d, "p_w1_single")
    ref = run_stream(single, "ref", queue.Queue())
    p1 = create(s1_d, "p_w1_s1")
    p0 = create(s0_d, "p_w1_s0")
    # the registrar's "add" of stage 1 as seen by stage 0 (rank tag: a hop over the data plane)
    from aiko_services_amd.runtime.actor import ActorTopic
    p0._post_message(ActorTopic.IN, "_pipeline_element_change_handler",
                     ["add", [p1.topic_path, "p_w1_s1", "pipeline:0", "mqtt", "test", ["rank=0"]]],
                     target_function=p0._pipeline_element_change_handler)
    deadline = time.time() + 30
    while p0.share.get("lifecycle") != "ready" and time.time() < deadline:
        time.sleep(0.02)
    got = run_stream(p0, "hop", queue.Queue())
    st = plane.stats()
    print("RESULT " + json.dumps({"ref": ref, "hop": got, "groups": p0.hop_groups, "hop_stats": st,
                                  "lanes": p0._frame_lanes()[0]}), flush=True)
    if not cpu:
        torch.cuda.synchronize()
    os._exit(0)


if __name__ == "__main__":
    main()
