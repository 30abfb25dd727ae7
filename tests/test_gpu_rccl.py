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


def test_pp_rank0_local_share_runs_two_lanes():
    """a stage ending in a remote element may run frame lanes, and rank 0's
    local share of the replicated ResNet stage runs in the enclosing frame's lane.  World-1 plan
    (stage 0 = decode + resize, stage 1 = ResNet-50 + top-k as rank 0's local share, 224²
    frames, B=256 as in config 3): the plan runs with one and with two lanes.  The lanes'
    speed-up is a benchmark, not a correctness property (scripts/lanes_ab.sh measures it)."""
    vals = {}
    for lanes in (1, 2):
        r = _torchrun("bench.py", "--parallel", "pp", "--gpus", "1", "--steps", "16", "--warmup", "4",
                      "--batch", "256", "--lanes", str(lanes), "--height", "224", "--width", "224")
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
        out = json.loads(lines[-1])
        assert out["config"]["local_share"] == 1.0 and out["config"]["stages"][1][0] == "ResNet50Classifier"
        vals[lanes] = out["value"]
    assert all(v > 0 for v in vals.values()), vals
