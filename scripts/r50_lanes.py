#!/usr/bin/env python3
"""ResNet-50 forward split into concurrent HIP-stream lanes: lanes -> ms per B-frame forward,
hipGraph-captured and eager (tiles autotuned per geometry first).

    python scripts/r50_lanes.py [--batch 256] [--lanes 1,2,3,4]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--lanes", default="1,2,3,4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--alt", default="1,2,3", help="alternate batches over this many streams")
    ap.add_argument("--stagger", default="none", help="comma list of block indices (none = no stagger)")
    a = ap.parse_args()
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    from aiko_services_amd.ops import require_native
    require_native()
    m = ResNet50(device="cuda")
    frames = torch.randint(0, 256, (a.batch, 224, 224, 3), dtype=torch.uint8, device="cuda")
    ref = None
    cfgs = [(int(n), None if st == "none" else int(st)) for n in a.lanes.split(",")
            for st in a.stagger.split(",") if int(n) > 1 or st == "none"]
    for n, st in cfgs:
        if a.batch % n:
            continue
        with C.autotune():
            out = m.logits_lanes(frames, n, frames=True, stagger=st)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.float().clone()
        err = (out.float() - ref).abs().max().item()
        eager = timed(lambda: m.logits_lanes(frames, n, frames=True, stagger=st), a.iters)
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.logits_lanes(frames, n, frames=True, stagger=st)
            with torch.cuda.graph(g, stream=s):
                m.logits_lanes(frames, n, frames=True, stagger=st)
        torch.cuda.current_stream().wait_stream(s)
        ms = timed(g.replay, a.iters)
        print(f"lanes={n} stagger={st}  graph {ms:7.3f} ms {a.batch / ms * 1e3:9.0f} frames/s   eager {eager:7.3f} ms"
              f"  max|d|={err:.3g}", flush=True)
        del g
    # alternate whole batches between K streams (each with its own workspace and graph)
    for k in (int(v) for v in a.alt.split(",") if v):
        graphs, streams = [], []
        for i in range(k):
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(st):
                m.logits(frames, tag=f"a{i}.")
                with torch.cuda.graph(g, stream=st):
                    m.logits(frames, tag=f"a{i}.")
            torch.cuda.current_stream().wait_stream(st)
            graphs.append(g)
            streams.append(st)
        torch.cuda.synchronize()
        cur = torch.cuda.current_stream()

        def run():
            for i in range(k):
                with torch.cuda.stream(streams[i]):
                    graphs[i].replay()
            for st in streams:
                cur.wait_stream(st)
        ms = timed(run, a.iters) / k
        print(f"alternate streams={k}  {ms:7.3f} ms/batch {a.batch / ms * 1e3:9.0f} frames/s", flush=True)


if __name__ == "__main__":
    main()
