"""the ENGINE's remote-hop path on a real GPU at world 1 — two stage
Pipelines joined over the loopback link with 2 frame lanes, hop_batch 4 and 2 credits, frames
queued for credits and dispatched in groups from other lanes / the event loop, group
responses flushed — must give the single-stage outputs bit for bit; with the hop plane's
cross-stream ordering stubbed out (``--no-order``) the same run must NOT (negative control:
the test would otherwise prove nothing).  Driver: ``tests/native/hop_engine_world1.py``."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "native", "hop_engine_world1.py"), *args],
                       cwd=ROOT, capture_output=True, text=True, timeout=150)
    m = re.search(r"RESULT (\{.*\})", r.stdout)
    assert m, (r.returncode, r.stdout[-3000:], r.stderr[-3000:])
    return json.loads(m.group(1))


def test_engine_hop_path_world1_matches_single_stage():
    res = _run()
    assert res["lanes"] == 2 and res["groups"] > 0, res            # frames really left in groups
    assert len(res["ref"]) == 24 and res["hop"] == res["ref"], res


def test_engine_hop_path_without_ordering_is_caught():
    res = _run("--no-order")
    assert len(res["ref"]) == 24
    assert res["hop"] != res["ref"], "stubbing HopPlane._order_after changed nothing: the test is blind"
