#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 image-classification pipeline, frames/s (whole node) + p50.

BASELINE.json metric "frames/sec (whole node) + p50 latency, ResNet-50 pipeline at 1/2/4/8
MI355X".  Every rank (one process per GPU, launched by torch.distributed.run) runs the aiko
Pipeline ``(SyntheticFrames ResNet50Classifier ClassifierTopK)`` — frames produced in HBM by
the synthetic decode stage, ResNet-50 bf16 on the HIP igemm/MFMA kernels, softmax/top-5 kernel,
results all-gathered over RCCL (data parallel, weak scaling: ``--batch`` frames per GPU per
step) and copied to pinned host memory.  Each step is one ``Pipeline.process_frame`` through
the aiko engine (graph walk, swag hand-off, metrics, response queue) — no work is skipped.

Timing: W untimed warmup steps, then exactly K steps bracketed by barrier +
torch.cuda.synchronize() on both sides; the elapsed time is the MAX over ranks.  p50 latency
is per batch, from submission to the top-5 results being available on the host.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import queue
import statistics
import sys
import time
from collections import deque

os.environ.setdefault("AIKO_MQTT_DISABLE", "1")      # data-plane bench: no broker needed
os.environ.setdefault("AIKO_LOG_MQTT", "false")
os.environ.setdefault("AIKO_LOG_LEVEL", "WARNING")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

METRIC = "frames/sec (whole node) + p50 latency, ResNet-50 pipeline at 1/2/4/8 MI355X"
ELEMENTS = "aiko_services_amd.elements.gpu.vision"


def definition(batch: int, graph: bool, height: int, width: int, lanes: int = 1) -> dict:
    def el(name, inputs, outputs, params=None):
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in inputs],
                "output": [{"name": n, "type": "tensor"} for n in outputs],
                "parameters": params or {}, "deploy": {"local": {"module": ELEMENTS}}}
    return {
        "version": 0, "name": "p_resnet50_bench", "runtime": "python",
        "graph": ["(SyntheticFrames ResNet50Classifier ClassifierTopK)"],
        "parameters": {"gpu_lanes": lanes},
        "elements": [
            el("SyntheticFrames", [], ["images", "t_submit"],
               {"batch": batch, "height": height, "width": width, "pool": 4}),
            el("ResNet50Classifier", ["images"], ["logits"], {"graph": graph}),
            el("ClassifierTopK", ["logits", "t_submit"], ["topk"], {"k": 5, "gather": True}),
        ],
    }


DETECT = "aiko_services_amd.elements.gpu.detect"


def yolo_definition(batch: int, graph: bool, height: int, width: int, fanout: str, lanes: int = 1) -> dict:
    """BASELINE config 4: ingest rank decodes the node's frames, RCCL fan-out, YOLOv8-n +
    NMS kernels per GPU, RCCL all-gather of fixed-size detections."""
    def el(name, module, inputs, outputs, params):
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in inputs],
                "output": [{"name": n, "type": "tensor"} for n in outputs],
                "parameters": params, "deploy": {"local": {"module": module}}}
    return {
        "version": 0, "name": "p_yolov8n_dp", "runtime": "python",
        "graph": ["(SyntheticFrames FrameFanout YoloDetector DetectionsGather)"],
        "parameters": {"gpu_lanes": lanes},
        "elements": [
            el("SyntheticFrames", ELEMENTS, [], ["images", "t_submit"],
               {"batch": batch, "height": height, "width": width, "pool": 2, "global": True}),
            el("FrameFanout", DETECT, ["images"], ["images"],
               {"mode": fanout, "batch": batch, "height": height, "width": width}),
            el("YoloDetector", DETECT, ["images"], ["detections", "counts"], {"graph": graph, "scale": "n"}),
            el("DetectionsGather", DETECT, ["detections", "counts", "t_submit"], ["detections"], {}),
        ],
    }


SPEECH = "aiko_services_amd.elements.gpu.speech"
YOLO_METRIC = "frames/sec (whole node) + p50 latency, YOLOv8-n data-parallel detection pipeline (BASELINE config 4)"
WHISPER_METRIC = "30 s audio windows/sec (whole node) + p50 latency, Whisper encoder fp8 on streamed chunks"


def whisper_definition(streams: int, graph: bool, size: str, chunk: float, window: float,
                       lanes: int = 1, transcribe: int = 0) -> dict:
    """BASELINE config 5: streamed audio chunks -> per-stream sliding window on the GPU ->
    log-mel + Whisper encoder (fp8 linears) -> pooled features to the host."""
    def el(name, inputs, outputs, params):
        return {"name": name, "input": [{"name": n, "type": "tensor"} for n in inputs],
                "output": [{"name": n, "type": "tensor"} for n in outputs],
                "parameters": params, "deploy": {"local": {"module": SPEECH}}}
    if transcribe:      # speech-to-text: greedy decoding of ``transcribe`` tokens per window
        return {
            "version": 0, "name": "p_whisper_asr", "runtime": "python",
            "graph": ["(AudioChunks AudioWindow WhisperEncoder WhisperTranscribe)"],
            "parameters": {"gpu_lanes": lanes},
            "elements": [
                el("AudioChunks", [], ["audio", "t_submit"], {"streams": streams, "chunk": chunk}),
                el("AudioWindow", ["audio"], ["audio"], {"window": window}),
                el("WhisperEncoder", ["audio"], ["features"], {"size": size, "graph": graph}),
                el("WhisperTranscribe", ["features", "t_submit"], ["transcript", "text"],
                   {"size": size, "graph": graph, "max_tokens": transcribe, "stop_early": False,
                    "defer_text": True}),
            ],
        }
    return {
        "version": 0, "name": "p_whisper_encoder", "runtime": "python",
        "graph": ["(AudioChunks AudioWindow WhisperEncoder FeatureSink)"],
        "parameters": {"gpu_lanes": lanes},
        "elements": [
            el("AudioChunks", [], ["audio", "t_submit"], {"streams": streams, "chunk": chunk}),
            el("AudioWindow", ["audio"], ["audio"], {"window": window}),
            el("WhisperEncoder", ["audio"], ["features"], {"size": size, "graph": graph}),
            el("FeatureSink", ["features", "t_submit"], ["embedding"], {}),
        ],
    }


def pp_definition(batch: int, graph: bool, height: int, width: int, world: int) -> dict:
    """BASELINE config 3: decode -> resize/normalise -> ResNet-50 -> post-process, one stage per
    GPU (``deploy.local.stage`` = i * world // 4, so fewer GPUs fold neighbouring stages)."""
    d = definition(batch, graph, height, width)
    d["name"] = "p_resnet50_pp"
    d["graph"] = ["(SyntheticFrames ImagePreprocess ResNet50Classifier ClassifierTopK)"]
    pre = {"name": "ImagePreprocess", "input": [{"name": "images", "type": "tensor"}],
           "output": [{"name": "images", "type": "tensor"}], "parameters": {"image_size": 224},
           "deploy": {"local": {"module": ELEMENTS}}}
    d["elements"].insert(1, pre)
    d["elements"][3]["parameters"]["gather"] = False
    for i, e in enumerate(d["elements"]):
        e["deploy"]["local"]["stage"] = i * world // 4
    return d


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256, help="frames per GPU per step")
    ap.add_argument("--height", type=int, default=224)
    ap.add_argument("--width", type=int, default=224)
    ap.add_argument("--no-graph", action="store_true", help="disable hipGraph capture")
    ap.add_argument("--depth", type=int, default=2, help="batches in flight")
    ap.add_argument("--lanes", type=int, default=2,
                    help="frame lanes: successive batches alternate over this many HIP "
                         "streams with private workspaces (gpu/lanes.py)")
    ap.add_argument("--model", choices=["resnet50", "yolov8n", "whisper-small", "whisper-tiny", "whisper-base"],
                    default="resnet50",
                    help="resnet50: headline ResNet-50 pipeline (config 2/3); yolov8n: config 4; "
                         "whisper-*: config 5 (--batch = concurrent audio streams)")
    ap.add_argument("--chunk", type=float, default=5.0, help="(whisper) seconds of audio per chunk")
    ap.add_argument("--window", type=float, default=30.0, help="(whisper) encoder window seconds")
    ap.add_argument("--transcribe", type=int, default=0,
                    help="(whisper) decode this many tokens per window (speech-to-text) instead of pooling features")
    ap.add_argument("--fanout", choices=["scatter", "broadcast"], default="scatter",
                    help="(yolov8n) RCCL fan-out of the ingest rank's frame batch")
    ap.add_argument("--parallel", choices=["dp", "pp"], default="dp",
                    help="dp: every GPU runs the whole pipeline (config 2/headline); "
                         "pp: one pipeline stage per GPU over RCCL P2P (config 3)")
    a = ap.parse_args(argv)
    explicit_hw = "--height" in (argv or sys.argv)
    if (a.parallel == "pp" or a.model == "yolov8n") and not explicit_hw:
        a.height, a.width = 480, 640          # configs 3/4 decode VGA video frames
    if a.model == "yolov8n" and "--batch" not in (argv or sys.argv):
        a.batch = 64
    if a.model.startswith("whisper") and "--batch" not in (argv or sys.argv):
        a.batch = 16

    from aiko_services_amd.parallel import dist as D
    D.init()
    ws, rank = D.world_size(), D.rank()
    if ws != a.gpus and rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {ws}", file=sys.stderr)
    from aiko_services_amd.gpu.device import select_device
    device = select_device()

    from aiko_services_amd.ops import require_native
    require_native()
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    from aiko_services_amd.pipeline.engine import PipelineImpl

    if a.parallel == "pp":
        return run_pp(a, device)
    metric, unit = METRIC, "frames/s"
    if a.model.startswith("whisper"):
        size = a.model.split("-", 1)[1]
        d = parse_pipeline_definition_dict(whisper_definition(a.batch, not a.no_graph, size, a.chunk, a.window,
                                                              a.lanes, a.transcribe))
        result_key = "transcript" if a.transcribe else "embedding"
        model_cfg = {"model": f"whisper-{size}" + ("-asr" if a.transcribe else "-encoder"),
                     "weights": "fp8 e4m3 (per-channel)", "decode_tokens": a.transcribe,
                     "chunk_s": a.chunk, "window_s": a.window, "streams": a.batch,
                     "pipeline": d.graph[0], "gpu_lanes": a.lanes}
        metric, unit = WHISPER_METRIC, "windows/s"
    elif a.model == "yolov8n":
        d = parse_pipeline_definition_dict(yolo_definition(a.batch, not a.no_graph, a.height, a.width, a.fanout, a.lanes))
        result_key, model_cfg = "detections", {"model": "yolov8n", "image_size": [640, 640],
                                               "frame_size": [a.height, a.width], "fanout": a.fanout,
                                               "pipeline": d.graph[0], "gpu_lanes": a.lanes}
        metric = YOLO_METRIC
    else:
        d = parse_pipeline_definition_dict(definition(a.batch, not a.no_graph, a.height, a.width, a.lanes))
        result_key, model_cfg = "topk", {"model": "resnet50", "image_size": [a.height, a.width],
                                         "pipeline": "(SyntheticFrames ResNet50Classifier ClassifierTopK)",
                                         "gpu_lanes": a.lanes}
    responses: queue.Queue = queue.Queue()
    pipeline = PipelineImpl.create_pipeline("<bench>", d, None, None, "bench", [], 0, None, 3600,
                                            queue_response=responses)
    frame_id = 0
    inflight: deque = deque()
    latencies: list = []

    def step(record):
        nonlocal frame_id
        pipeline.process_frame({"stream_id": "bench", "frame_id": frame_id}, {})
        frame_id += 1
        info, out = responses.get_nowait()
        if info["state"] != 0:
            raise RuntimeError(f"pipeline frame failed: {info} {out}")
        inflight.append((out[result_key], record))
        while len(inflight) > a.depth:
            res, rec = inflight.popleft()
            res.wait()
            if rec:
                latencies.append(res.latency)

    def drain(record=True):
        while inflight:
            res, rec = inflight.popleft()
            res.wait()
            if rec and record:
                latencies.append(res.latency)

    for _ in range(a.warmup):
        step(False)
    drain(False)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    drain()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    t = torch.tensor([elapsed, statistics.median(latencies) if latencies else 0.0],
                     dtype=torch.float64, device=device)
    D.all_reduce_max(t)
    elapsed, p50 = float(t[0]), float(t[1])
    frames = ws * a.batch * a.steps
    fps = frames / elapsed
    if rank == 0:
        out = {
            "metric": metric, "value": round(fps, 1), "unit": unit, "n_gpus": ws,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp8 linears / bf16 conv+attention" if a.model.startswith("whisper") else "bf16",
            "data": (f"synthetic ({a.batch} streams of {a.chunk:g} s 16 kHz chunks generated in HBM; random-init weights)"
                     if a.model.startswith("whisper") else
                     f"synthetic (random uint8 {a.height}x{a.width} frames generated in HBM; random-init weights)"),
            "p50_latency_ms": round(p50 * 1e3, 3),
            "config": dict({"global_batch": ws * a.batch, "seq_len": None, "per_gpu_batch": a.batch,
                            "parallelism": f"dp{ws}", "hipgraph": not a.no_graph}, **model_cfg),
        }
        if a.model.startswith("whisper"):
            out["audio_seconds_per_s"] = round(ws * a.batch * a.chunk * a.steps / elapsed, 1)
            if a.transcribe:
                out["decoded_tokens_per_s"] = round(ws * a.batch * a.transcribe * a.steps / elapsed, 1)
        print(json.dumps(out), flush=True)
    D.barrier()
    D.destroy()


def run_pp(a, device):
    """Config 3: the stages of one pipeline spread over the GPUs; frames/s counted at the last
    stage (each frame batch is processed once by the whole node)."""
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel.pipeline_parallel import PipelineParallelRunner
    from aiko_services_amd.pipeline.definition import parse_pipeline_definition_dict
    ws, rank = D.world_size(), D.rank()
    d = parse_pipeline_definition_dict(pp_definition(a.batch, not a.no_graph, a.height, a.width, ws))
    D.barrier()
    runner = PipelineParallelRunner(d, device=device, depth=2, stream_id="bench")
    inflight: deque = deque()
    latencies: list = []

    def step(record):
        r = runner.step({})
        if r is None:
            return
        info, out = r
        if info["state"] != 0:
            raise RuntimeError(f"pipeline frame failed: {info} {out}")
        inflight.append((out["topk"], record))
        while len(inflight) > a.depth:
            res, rec = inflight.popleft()
            res.wait()
            if rec:
                latencies.append(res.latency)

    def drain(record=True):
        while inflight:
            res, rec = inflight.popleft()
            res.wait()
            if rec and record:
                latencies.append(res.latency)

    for _ in range(a.warmup):
        step(False)
    drain(False)
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    runner.finish()
    drain()
    torch.cuda.synchronize()
    D.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, statistics.median(latencies) if latencies else 0.0],
                     dtype=torch.float64, device=device)
    D.all_reduce_max(t)
    elapsed, p50 = float(t[0]), float(t[1])
    fps = a.batch * a.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": METRIC, "value": round(fps, 1), "unit": "frames/s", "n_gpus": ws,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
            "data": f"synthetic (random uint8 {a.height}x{a.width} frames generated in HBM; random-init weights)",
            "p50_latency_ms": round(p50 * 1e3, 3),
            "config": {"model": "resnet50", "global_batch": a.batch, "seq_len": None,
                       "image_size": [224, 224], "frame_size": [a.height, a.width],
                       "per_gpu_batch": a.batch, "parallelism": f"pp{ws}", "hipgraph": not a.no_graph,
                       "stages": runner.stages,
                       "pipeline": "(SyntheticFrames ImagePreprocess ResNet50Classifier ClassifierTopK)"},
        }), flush=True)
    D.barrier()
    D.destroy()


if __name__ == "__main__":
    main()
