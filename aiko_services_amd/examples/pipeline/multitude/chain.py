"""Multi-process pipeline chain load test (the reference's "multitude" small / large runs:
``examples/pipeline/multitude/pipeline_small_{a,b,c}.json`` — 3 processes — and
``pipeline_large_0{00..90}.json`` — 10 processes x 11 elements, driven by ``run_*.sh``).

Generates ``--processes`` pipeline definitions; stage k holds ``--elements`` local ``PE_Add``
elements followed by a remote element bound (through the registrar) to stage k + 1.  The
parent (stage 0) pushes ``--frames`` frames with a window of frames in flight; every frame
crosses every process boundary twice (request and response) as S-expression messages.

    python -m aiko_services_amd.examples.pipeline.multitude.chain --processes 3 --elements 3
    python -m aiko_services_amd.examples.pipeline.multitude.chain --processes 10 --elements 11

Prints one JSON line: frames/s and p50 / p99 end-to-end latency.
"""
from __future__ import annotations

import argparse
import json
import os
import tempfile

MODULE = "aiko_services_amd.examples.pipeline.multitude.elements"


def chain_definitions(processes: int, elements: int) -> list[dict]:
    defs = []
    for k in range(processes):
        names = [f"S{k}_E{j}" for j in range(elements)]
        elems = [{"name": n, "input": [{"name": "i", "type": "int"}], "output": [{"name": "i", "type": "int"}],
                  "deploy": {"local": {"module": "aiko_services_amd.examples.pipeline.elements",
                                       "class_name": "PE_Add"}}} for n in names]
        if k < processes - 1:
            names.append(f"S{k}_Next")
            elems.append({"name": f"S{k}_Next", "input": [{"name": "i", "type": "int"}],
                          "output": [{"name": "i", "type": "int"}],
                          "deploy": {"remote": {"module": MODULE,
                                                "service_filter": {"name": f"p_chain_{k + 1}"}}}})
        defs.append({"version": 0, "name": f"p_chain_{k}", "runtime": "python",
                     "graph": ["(" + " ".join(names) + ")"], "elements": elems})
    return defs


def run(processes=3, elements=3, frames=1000, window=8, timeout=120.0) -> dict:
    from ....tools.echo_bench import orchestrate
    with tempfile.TemporaryDirectory(prefix="aiko_chain_") as tmp:
        paths = []
        for d in chain_definitions(processes, elements):
            path = os.path.join(tmp, d["name"] + ".json")
            with open(path, "w") as f:
                json.dump(d, f)
            paths.append(path)
        res = orchestrate(frames, window, timeout, parent=paths[0], children=paths[1:],
                          expect=processes * elements)
    res.update({"processes": processes, "elements_per_process": elements})
    return res


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--processes", type=int, default=3)
    ap.add_argument("--elements", type=int, default=3)
    ap.add_argument("--frames", type=int, default=1000)
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--timeout", type=float, default=120.0)
    a = ap.parse_args(argv)
    res = run(a.processes, a.elements, a.frames, a.window, a.timeout)
    res["metric"] = "multi-process pipeline chain frames/s over MQTT"
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
