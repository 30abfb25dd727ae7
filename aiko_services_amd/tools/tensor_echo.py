"""Tensor round trip through a plain ``deploy.remote`` element (no ``parallel`` block, no RCCL
plan): arrays cross the MQTT control plane as binary tensor payloads
(``message/tensor_payload.py``) — the path of the reference's remote hop
(``/root/reference/src/aiko_services/main/pipeline.py:1080-1090``) when its inputs are arrays.

Topology: registrar process, child pipeline ``p_tensor_child`` (``TensorEcho``), parent pipeline
``p_tensor_parent`` ``(Tensor_Remote)``.  Every frame sends a float32 ``[4, 3, 224, 224]``
tensor ``x`` (on ``--device``) and a uint8 ``[4, 224, 224, 3]`` ndarray ``u``; the response must
hold them bit-exact, plus ``x2 = 2 x`` and ``u_sum`` computed on the far side.

    python -m aiko_services_amd.tools.tensor_echo [--frames 8] [--device cpu|cuda]

Prints one JSON line (frames, MB/s of array payload each way, mismatches).
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import subprocess
import sys
import threading
import time
import uuid
from pathlib import Path

DEFS = Path(__file__).resolve().parent.parent / "examples" / "pipeline" / "definitions"


def make_frame(frame_id: int, device: str):
    import numpy as np
    import torch
    g = torch.Generator().manual_seed(1000 + frame_id)
    x = torch.randn(4, 3, 224, 224, generator=g, dtype=torch.float32).to(device)
    u = np.random.default_rng(frame_id).integers(0, 256, size=(4, 224, 224, 3), dtype=np.uint8)
    return x, u


def _parent(frames: int, device: str, timeout: float):
    import numpy as np
    import torch

    import aiko_services_amd as aiko
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition
    from aiko_services_amd.pipeline.engine import PipelineImpl
    from aiko_services_amd.runtime import event

    q: queue.Queue = queue.Queue()
    path = str(DEFS / "tensor_remote_parent.json")
    pipeline = PipelineImpl.create_pipeline(path, parse_pipeline_definition(path), None, None, "1", [], 0,
                                            None, 600, queue_response=q)
    result = {"frames": 0, "mismatches": [], "device": device}

    def driver():
        deadline = time.time() + timeout
        while "1" not in pipeline.stream_leases or pipeline.share.get("lifecycle") != "ready":
            if time.time() > deadline:
                result["error"] = "remote pipeline not discovered"
                break
            time.sleep(0.05)
        sent = {}
        t0 = time.perf_counter()
        if "error" not in result:
            for i in range(frames):
                x, u = make_frame(i, device)
                sent[i] = (x, u)
                pipeline.create_frame({"stream_id": "1", "frame_id": i}, {"x": x, "u": u})
            while result["frames"] < frames:
                try:
                    info, data = q.get(timeout=max(1.0, deadline - time.time()))
                except queue.Empty:
                    result["error"] = f"timeout after {result['frames']} frames"
                    break
                fid = int(info["frame_id"])
                x, u = sent.pop(fid)
                rx, ru, rx2 = data.get("x"), data.get("u"), data.get("x2")
                ok = (isinstance(rx, torch.Tensor) and rx.dtype == x.dtype and rx.device.type == x.device.type
                      and torch.equal(rx, x) and isinstance(rx2, torch.Tensor) and torch.equal(rx2, x * 2)
                      and isinstance(ru, np.ndarray) and ru.dtype == u.dtype and np.array_equal(ru, u)
                      and int(data.get("u_sum", -1)) == int(u.astype(np.int64).sum()))
                if not ok:
                    result["mismatches"].append(fid)
                result["device_in"] = data.get("device_in")
                result["frames"] += 1
        elapsed = time.perf_counter() - t0
        mb = frames * (4 * 3 * 224 * 224 * 4 + 4 * 224 * 224 * 3) / 1e6
        result["payload_mb_per_s"] = round(mb / elapsed, 1) if elapsed > 0 else None
        print("TENSOR_ECHO_RESULT " + json.dumps(result), flush=True)
        event.call_soon(aiko.process.terminate, 0)

    threading.Thread(target=driver, daemon=True).start()
    pipeline.run(mqtt_connection_required=True)


def orchestrate(frames=4, device="cpu", timeout=60.0, broker_port=None):
    from aiko_services_amd.message.mqtt_broker import start_broker_thread
    broker = None
    if broker_port is None:
        broker, broker_port = start_broker_thread("127.0.0.1", 0)
    env = dict(os.environ)
    env.update({"AIKO_MQTT_HOST": "127.0.0.1", "AIKO_MQTT_PORT": str(broker_port),
                "AIKO_NAMESPACE": f"tensor{uuid.uuid4().hex[:6]}", "AIKO_LOG_MQTT": "false",
                "AIKO_LOG_LEVEL": "WARNING", "AIKO_REGISTRAR_SEARCH_TIMEOUT": "0.3",
                "AIKO_MQTT_DISABLE": "0", "PYTHONPATH": str(DEFS.parents[3]) + os.pathsep + env.get("PYTHONPATH", "")})
    procs = []
    try:
        procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.tools.registrar"], env=env))
        time.sleep(0.5)
        procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.pipeline.cli", "create",
                                       str(DEFS / "tensor_remote_child.json")], env=env))
        cmd = [sys.executable, "-m", "aiko_services_amd.tools.tensor_echo", "--role", "parent",
               "--frames", str(frames), "--device", device, "--timeout", str(timeout)]
        parent = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout + 60)
        for line in parent.stdout.splitlines():
            if line.startswith("TENSOR_ECHO_RESULT "):
                return json.loads(line[len("TENSOR_ECHO_RESULT "):])
        return {"error": f"parent rc={parent.returncode}: {parent.stderr[-3000:]}"}
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(5)
            except subprocess.TimeoutExpired:
                p.kill()
        if broker is not None:
            broker.stop()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--role", default="orchestrate", choices=["orchestrate", "parent"])
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--timeout", type=float, default=60.0)
    a = ap.parse_args(argv)
    if a.role == "parent":
        _parent(a.frames, a.device, a.timeout)
    else:
        print(json.dumps(orchestrate(a.frames, a.device, a.timeout)), flush=True)


if __name__ == "__main__":
    main()
