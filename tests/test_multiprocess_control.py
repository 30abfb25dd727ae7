"""Multi-process control plane over the in-repo MQTT broker (multi-node emulation the way the
reference does it: several processes on one host, isolated by AIKO_NAMESPACE).

* BASELINE config 1: two-process echo pipeline (registrar discovery + remote PipelineElement
  + process_frame / process_frame_response), compared with the reference's 50 frames/s;
* registrar directory: dashboard snapshot lists services; process LWT removes them;
* storage actor request/response through discovery.
"""
import os
import subprocess
import sys
import time
import uuid

import pytest

from aiko_services_amd.message.mqtt_broker import start_broker_thread

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def cluster():
    broker, port = start_broker_thread("127.0.0.1", 0)
    env = dict(os.environ)
    env.update({"AIKO_MQTT_HOST": "127.0.0.1", "AIKO_MQTT_PORT": str(port),
                "AIKO_NAMESPACE": f"t{uuid.uuid4().hex[:8]}", "AIKO_LOG_MQTT": "false",
                "AIKO_LOG_LEVEL": "WARNING", "AIKO_REGISTRAR_SEARCH_TIMEOUT": "0.3",
                "AIKO_MQTT_DISABLE": "0", "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
    procs = []

    def spawn(*args):
        p = subprocess.Popen([sys.executable, *args], env=env, cwd=ROOT,
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        procs.append(p)
        return p

    def run(*args, timeout=30):
        return subprocess.run([sys.executable, *args], env=env, cwd=ROOT, capture_output=True, text=True,
                              timeout=timeout)
    yield {"port": port, "env": env, "spawn": spawn, "run": run, "broker": broker}
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(5)
        except subprocess.TimeoutExpired:
            p.kill()
    broker.stop()


def test_echo_pipeline_beats_reference(cluster):
    from aiko_services_amd.tools.echo_bench import orchestrate
    res = orchestrate(frames=300, window=4, timeout=40, broker_port=cluster["port"])
    assert "error" not in res, res
    assert res["frames"] == 300
    assert res["frames_per_s"] > 50, res      # reference ceiling: 50 frames/s


def _snapshot(cluster, service=None, expect=(), timeout=40):   # generous: returns as soon as seen
    deadline = time.time() + timeout
    out = ""
    while time.time() < deadline:
        args = ["-m", "aiko_services_amd.tools.dashboard", "--snapshot", "--timeout", "3"]
        if service:
            args += ["--service", service]
        out = cluster["run"](*args).stdout
        if all(e in out for e in expect):
            return out
        time.sleep(0.3)
    return out


def test_registrar_directory_and_lwt(cluster):
    cluster["spawn"]("-m", "aiko_services_amd.tools.registrar")
    time.sleep(0.8)
    store = cluster["spawn"]("-m", "aiko_services_amd.tools.storage", "start", ":memory:")
    out = _snapshot(cluster, expect=("registrar", "storage"))
    assert "registrar" in out and "storage" in out, out
    out = _snapshot(cluster, service="registrar", expect=("service_count",))
    assert "lifecycle = primary" in out and "service_count" in out, out
    # abnormal termination -> broker fires the process LWT -> registrar removes its services
    store.kill()
    deadline = time.time() + 15
    while time.time() < deadline:
        out = _snapshot(cluster, expect=("registrar",), timeout=5)
        if "storage" not in out:
            break
        time.sleep(0.3)
    assert "storage" not in out, out


def test_storage_request_response(cluster):
    cluster["spawn"]("-m", "aiko_services_amd.tools.registrar")
    time.sleep(0.8)
    cluster["spawn"]("-m", "aiko_services_amd.tools.storage", "start", ":memory:")
    res = cluster["run"]("-m", "aiko_services_amd.tools.storage", "test_request", "hello_world", timeout=30)
    assert "Response: [('hello_world', [])]" in res.stdout, res.stdout + res.stderr


def test_aloha_honua_actor_over_mqtt(cluster):
    """Hello-world actor (X1): remote call published as an S-expression on its /in topic."""
    cluster["spawn"]("-m", "aiko_services_amd.tools.registrar")
    time.sleep(0.8)
    actor = cluster["spawn"]("-m", "aiko_services_amd.examples.aloha_honua.aloha_honua_0")
    topic = None
    deadline = time.time() + 15
    while time.time() < deadline and topic is None:
        line = actor.stdout.readline()
        if line.startswith("MQTT topic:"):
            topic = line.split(":", 1)[1].strip()
    assert topic, "actor did not report its topic"
    out = _snapshot(cluster, expect=("aloha_honua",))
    assert "aloha_honua" in out
    for name in ("Pele", "Hiiaka"):
        r = cluster["run"]("-m", "aiko_services_amd.tools.mqtt", "pub", topic, f"(aloha {name})")
        assert r.returncode == 0, r.stderr
    out = _snapshot(cluster, service="aloha_honua", expect=("greetings = 2",))
    assert "greetings = 2" in out, out


def test_multitude_chain_three_processes():
    """The reference's multitude load test topology: a chain of pipeline processes, each
    stage's last element remote-bound (via the registrar) to the next process."""
    from aiko_services_amd.examples.pipeline.multitude.chain import run
    res = run(processes=3, elements=2, frames=100, window=4, timeout=60)
    assert "error" not in res, res
    assert res["frames"] == 100 and res["frames_per_s"] > 50


def test_tensor_payload_through_plain_remote(cluster):
    """A float32 [4, 3, 224, 224] tensor and a uint8 ndarray cross a plain ``deploy.remote``
    hop (registrar-discovered child, no ``parallel`` block) and come back bit-exact."""
    from aiko_services_amd.tools.tensor_echo import orchestrate
    res = orchestrate(frames=3, device="cpu", timeout=60, broker_port=cluster["port"])
    assert "error" not in res, res
    assert res["frames"] == 3 and res["mismatches"] == [], res
    assert res["device_in"] == "cpu"


def test_echo_pipeline_over_websockets():
    """Config 1 (two-process echo pipeline + registrar) with every process on MQTT over
    WebSockets (AIKO_MQTT_TRANSPORT=websockets; reference main/message/mqtt.py:87,108)."""
    from aiko_services_amd.tools.echo_bench import orchestrate
    broker, _port = start_broker_thread("127.0.0.1", 0, ws_port=0)
    try:
        res = orchestrate(frames=200, window=4, timeout=40, broker_port=broker.ws_port,
                          extra_env={"AIKO_MQTT_TRANSPORT": "websockets"})
    finally:
        broker.stop()
    assert "error" not in res, res
    assert res["frames"] == 200 and res["frames_per_s"] > 50, res
