"""BASELINE config 1: two-process echo pipeline over the MQTT control plane (CPU only).

Topology (all on one host, own broker):  registrar process, child pipeline process
``p_echo_child`` (``Echo_B``), parent pipeline process ``p_echo_parent``
``(Echo_A Echo_Remote Echo_C)`` where ``Echo_Remote`` is discovered through the registrar.
Every frame makes the round trip parent -> child -> parent as S-expression ``process_frame``
/ ``process_frame_response`` messages — the same plumbing the reference's multitude load test
measures (≤ 50 frames/s there).

    python -m aiko_services_amd.tools.echo_bench [--frames 2000] [--window 8]

Prints one JSON line: frames/s, p50 / p99 round-trip latency.
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import statistics
import subprocess
import sys
import threading
import time
import uuid
from pathlib import Path

DEFS = Path(__file__).resolve().parent.parent / "examples" / "pipeline" / "definitions"


def _parent(frames: int, window: int, timeout: float, definition: str | None = None, expect: int = 3):
    import aiko_services_amd as aiko
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition
    from aiko_services_amd.pipeline.engine import PipelineImpl
    from aiko_services_amd.runtime import event

    q: queue.Queue = queue.Queue()
    path = definition or str(DEFS / "echo_parent.json")
    definition = parse_pipeline_definition(path)
    pipeline = PipelineImpl.create_pipeline(path, definition, None, None, "1", [], 0, None, 600,
                                            queue_response=q)
    result = {}

    def driver():
        deadline = time.time() + timeout
        while "1" not in pipeline.stream_leases:
            if time.time() > deadline:
                result["error"] = "remote pipeline not discovered"
                aiko.process.terminate(1)
                return
            time.sleep(0.02)
        sent, t_sent, rtts = 0, {}, []
        t0 = time.perf_counter()
        while len(rtts) < frames:
            while sent < frames and sent - len(rtts) < window:
                t_sent[sent] = time.perf_counter()
                pipeline.create_frame({"stream_id": "1", "frame_id": sent}, {"i": 0})
                sent += 1
            try:
                info, data = q.get(timeout=max(1.0, deadline - time.time()))
            except queue.Empty:
                result["error"] = f"timeout after {len(rtts)} frames"
                break
            rtts.append(time.perf_counter() - t_sent.pop(int(info["frame_id"])))
            if int(data.get("i", -1)) != expect:
                result["error"] = f"bad echo payload {data}"
        elapsed = time.perf_counter() - t0
        if rtts:
            rtts.sort()
            result.update({"frames": len(rtts), "frames_per_s": len(rtts) / elapsed,
                           "p50_ms": statistics.median(rtts) * 1e3,
                           "p99_ms": rtts[min(len(rtts) - 1, int(0.99 * len(rtts)))] * 1e3,
                           "window": window})
        print("ECHO_RESULT " + json.dumps(result), flush=True)
        event.call_soon(aiko.process.terminate, 0)

    threading.Thread(target=driver, daemon=True).start()
    pipeline.run(mqtt_connection_required=True)


def orchestrate(frames=2000, window=8, timeout=60.0, broker_port=None, parent=None, children=None,
                expect=3, extra_env=None):
    """Registrar + child pipeline processes + a parent driving ``frames`` through the chain."""
    from aiko_services_amd.message.mqtt_broker import start_broker_thread
    broker = None
    if broker_port is None:
        broker, broker_port = start_broker_thread("127.0.0.1", 0)
    env = dict(os.environ)
    env.update({"AIKO_MQTT_HOST": "127.0.0.1", "AIKO_MQTT_PORT": str(broker_port),
                "AIKO_NAMESPACE": f"echo{uuid.uuid4().hex[:6]}", "AIKO_LOG_MQTT": "false",
                "AIKO_LOG_LEVEL": "WARNING", "AIKO_REGISTRAR_SEARCH_TIMEOUT": "0.3",
                "AIKO_MQTT_DISABLE": "0", "PYTHONPATH": str(DEFS.parents[3]) + os.pathsep + env.get("PYTHONPATH", "")})
    env.update(extra_env or {})          # e.g. AIKO_MQTT_TRANSPORT=websockets
    procs = []
    try:
        procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.tools.registrar"], env=env))
        time.sleep(0.5)
        for child in children or [str(DEFS / "echo_child.json")]:
            procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.pipeline.cli", "create",
                                           str(child)], env=env))
        cmd = [sys.executable, "-m", "aiko_services_amd.tools.echo_bench", "--role", "parent",
               "--frames", str(frames), "--window", str(window), "--timeout", str(timeout),
               "--expect", str(expect)]
        if parent:
            cmd += ["--definition", str(parent)]
        parent = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout + 30)
        for line in parent.stdout.splitlines():
            if line.startswith("ECHO_RESULT "):
                return json.loads(line[len("ECHO_RESULT "):])
        return {"error": f"parent rc={parent.returncode}: {parent.stderr[-2000:]}"}
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
    ap.add_argument("--frames", type=int, default=2000)
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--timeout", type=float, default=60.0)
    ap.add_argument("--definition", default=None, help="(parent role) parent pipeline definition")
    ap.add_argument("--expect", type=int, default=3, help="(parent role) expected 'i' at the end")
    a = ap.parse_args(argv)
    if a.role == "parent":
        _parent(a.frames, a.window, a.timeout, a.definition, a.expect)
    else:
        res = orchestrate(a.frames, a.window, a.timeout)
        res.update({"metric": "two-process echo pipeline frames/s over MQTT (config 1)",
                    "reference_ceiling_frames_per_s": 50})
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
