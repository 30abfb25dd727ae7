"""Micro-benchmark: ResNet-50 on aiko HIP kernels vs the same network on torch/MIOpen.

Per-layer times (our igemm kernel vs F.conv2d channels_last bf16 on identical shapes) and the
whole forward (eager and hipGraph-captured).  Writes JSON to --out.

    python scripts/bench_model.py --batch 256 --out gpurun_out/bench_model.json
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--layers", action="store_true", help="per-layer comparison")
    ap.add_argument("--out", default="gpurun_out/bench_model.json")
    a = ap.parse_args()
    from aiko_services_amd import ops
    ops.require_native()
    from aiko_services_amd.models.resnet50 import ResNet50
    from aiko_services_amd.ops import conv as C
    B = a.batch
    m = ResNet50(device="cuda")
    frames = torch.randint(0, 256, (B, 224, 224, 3), dtype=torch.uint8, device="cuda")
    res = {"batch": B, "gflop_per_image": m.flops_per_image() / 1e9}

    t = timeit(lambda: m(frames), a.iters)
    res["aiko_eager_ms"] = t
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m(frames)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        m(frames)
    t = timeit(g.replay, a.iters)
    res["aiko_graph_ms"] = t
    res["aiko_graph_fps"] = B / t * 1e3
    res["aiko_tflops"] = m.flops_per_image() * B / (t * 1e-3) / 1e12

    # torch / MIOpen reference network with the same folded weights, channels_last bf16
    def torch_forward(x):
        x = F.conv2d(x, wt["stem"], bt["stem"], stride=2, padding=3).relu_()
        x = F.max_pool2d(x, 3, 2, 1)
        for i, b in enumerate(m.blocks):
            t1 = F.conv2d(x, wt[f"{i}.1"], bt[f"{i}.1"]).relu_()
            t2 = F.conv2d(t1, wt[f"{i}.2"], bt[f"{i}.2"], stride=b.conv2.stride, padding=1).relu_()
            idn = F.conv2d(x, wt[f"{i}.d"], bt[f"{i}.d"], stride=b.down.stride) if b.down is not None else x
            x = (F.conv2d(t2, wt[f"{i}.3"], bt[f"{i}.3"]) + idn).relu_()
        x = x.mean((2, 3))
        return F.linear(x, wt["fc"], bt["fc"])

    def cl(w):
        return w.to("cuda", torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt, bt = {"stem": cl(m.stem.ref_weight)}, {"stem": m.stem.ref_bias.to("cuda", torch.bfloat16)}
    for i, b in enumerate(m.blocks):
        for tag, sp in (("1", b.conv1), ("2", b.conv2), ("3", b.conv3), ("d", b.down)):
            if sp is not None:
                wt[f"{i}.{tag}"] = cl(sp.ref_weight)
                bt[f"{i}.{tag}"] = sp.ref_bias.to("cuda", torch.bfloat16)
    wt["fc"] = m.fc.ref_weight.reshape(1000, 2048).to("cuda", torch.bfloat16)
    bt["fc"] = m.fc.ref_bias.to("cuda", torch.bfloat16)
    xin = torch.randn(B, 3, 224, 224, device="cuda", dtype=torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    with torch.no_grad():
        t = timeit(lambda: torch_forward(xin), a.iters)
    res["torch_miopen_ms"] = t
    res["torch_miopen_fps"] = B / t * 1e3

    if a.layers:
        rows = []
        H = 56
        x = torch.randn(B, H, H, 64, device="cuda", dtype=torch.bfloat16)
        shapes = []
        Hc = 56
        for i, b in enumerate(m.blocks):
            for tag, sp in (("conv1", b.conv1), ("conv2", b.conv2), ("conv3", b.conv3), ("down", b.down)):
                if sp is None:
                    continue
                Hin = Hc if tag in ("conv1", "conv2", "down") else b.conv2.out_hw(Hc, Hc)[0]
                shapes.append((f"b{i}.{tag}", sp, Hin))
            Hc = b.conv2.out_hw(Hc, Hc)[0]
        seen = set()
        for name, sp, Hin in shapes:
            key = (sp.cin, sp.cout, sp.R, sp.stride, Hin)
            if key in seen:
                continue
            seen.add(key)
            xi = torch.randn(B, Hin, Hin, sp.cin, device="cuda", dtype=torch.bfloat16)
            Ho, _ = sp.out_hw(Hin, Hin)
            res_t = torch.randn(B, Ho, Ho, sp.cout, device="cuda", dtype=torch.bfloat16) if name.endswith("conv3") else None
            out = torch.empty(B, Ho, Ho, sp.cout, device="cuda", dtype=torch.bfloat16)
            variants = {}
            for tile in ((128, 128), (128, 64), (64, 128), (64, 64)):
                if sp.cout % tile[1]:
                    continue
                variants[f"{tile[0]}x{tile[1]}"] = timeit(
                    lambda tile=tile: C.conv2d(xi, sp, residual=res_t, out=out, tile=tile), 10, 3)
            xt = xi.permute(0, 3, 1, 2)  # channels_last view
            wcl = cl(sp.ref_weight)
            tt = timeit(lambda: F.conv2d(xt, wcl, None, stride=sp.stride, padding=sp.pad), 10, 3)
            fl = sp.flops(B, Hin, Hin)
            best = min(variants.values())
            rows.append({"layer": name, "cin": sp.cin, "cout": sp.cout, "k": sp.R, "stride": sp.stride,
                         "hin": Hin, "ms": variants, "auto_tile": list(C.pick_tile(B * Ho * Ho, sp.cout)),
                         "torch_ms": tt, "best_tflops": fl / best / 1e9, "torch_tflops": fl / tt / 1e9})
            print(json.dumps(rows[-1]), flush=True)
        res["layers"] = rows
    print(json.dumps({k: v for k, v in res.items() if k != "layers"}, indent=1), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
