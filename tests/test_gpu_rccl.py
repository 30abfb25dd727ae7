"""RCCL readiness on one GPU: the ``nccl`` process-group paths, lane
all-gathers and the hop data plane under ``torch.distributed.run --nproc-per-node 1``, and the
config-3 actor-pipeline bench path (``bench.py --parallel pp``) end to end at world 1."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(*args, timeout=240):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=ROOT)
    return subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                           "--master-addr", "127.0.0.1", "--master-port", str(_port()), *args],
                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_rccl_world1_paths():
    r = _torchrun(os.path.join(ROOT, "tests", "native", "rccl_world1.py"))
    assert "RCCL_WORLD1_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])


def test_bench_pp_actor_path_world1():
    r = _torchrun("bench.py", "--parallel", "pp", "--gpus", "1", "--steps", "4", "--warmup", "2",
                  "--batch", "32")
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    out = json.loads(lines[-1])
    assert out["config"]["parallelism"] == "pp1" and out["value"] > 0
