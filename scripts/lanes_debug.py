#!/usr/bin/env python3
"""Debug: Whisper sliding-window pipeline outputs per frame, lanes 1 vs 2 (env decides the
graph admission policy); prints the pooled embeddings' checksums per frame."""
import os
import queue
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def run(d, frames):
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl
    q = queue.Queue()
    p = PipelineImpl.create_pipeline("<t>", parse_pipeline_definition_dict(d), None, None, "l", [], 0,
                                     None, 60, queue_response=q)
    outs = []
    for i in range(frames):
        p.process_frame({"stream_id": "l", "frame_id": i}, {})
        info, out = q.get_nowait()
        outs.append(next(iter(out.values())))
    return [r.wait()["pooled"].clone() for r in outs]


def main():
    os.environ.setdefault("AIKO_MQTT_DISABLE", "1")
    import bench
    graph = os.environ.get("DBG_GRAPH", "1") == "1"
    if os.environ.get("DBG_YOLO_FIRST"):
        for lanes in (1, 2):
            run_yolo = bench.yolo_definition(2, True, 240, 320, "scatter", lanes)
            from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
            from aiko_services_amd.pipeline.engine import PipelineImpl
            q = queue.Queue()
            p = PipelineImpl.create_pipeline("<y>", parse_pipeline_definition_dict(run_yolo), None, None, "l", [], 0,
                                             None, 60, queue_response=q)
            for i in range(5):
                p.process_frame({"stream_id": "l", "frame_id": i}, {})
                q.get_nowait()[1]
            del p
    for lanes in (1, 2):
        res = run(bench.whisper_definition(2, graph, "tiny", 2.0, 6.0, lanes), 6)
        print(f"lanes={lanes} graph={graph}:", " ".join(f"{float(r.double().sum()):.6f}" for r in res), flush=True)


if __name__ == "__main__":
    main()
