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
SETUP_FRAMES = 12     # >= frame-pool slots x lanes distinct (slot, lane) graphs, see main()
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
               {"batch": batch, "height": height, "width": width, "pool": 6}),
            el("ResNet50Classifier", ["images"], ["logits"], {"graph": graph}),
            el("ClassifierTopK", ["logits", "t_submit"], ["topk"], {"k": 5, "gather": True}),
        ],
    }


DETECT = "aiko_services_amd.elements.gpu.detect"


def host_ingest(d: dict) -> dict:
    """``--ingest host``: the source makes its frames in pinned HOST memory (a decoder's
    output) and a FrameUpload element brings each batch into an HBM FramePool slot on its own
    copy stream — the PCIe upload of configs 3/4 modelled on every rank."""
    d = json.loads(json.dumps(d))
    src = d["elements"][0]
    assert src["name"] == "SyntheticFrames"
    src["parameters"]["host"] = True
    src["parameters"].pop("global", None)
    up = {"name": "FrameUpload", "input": [{"name": "images", "type": "tensor"}],
          "output": [{"name": "images", "type": "tensor"}],
          "parameters": {"pool": src["parameters"].get("pool", 6)}, "deploy": {"local": {"module": ELEMENTS}}}
    d["elements"].insert(1, up)
    g = d["graph"][0]
    d["graph"] = [g.replace("(SyntheticFrames ", "(SyntheticFrames FrameUpload ", 1)]
    return d


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
               {"batch": batch, "height": height, "width": width, "pool": 4, "global": True}),
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


def pp_definition(batch: int, graph: bool, height: int, width: int, world: int, lanes: int = 1) -> dict:
    """BASELINE config 3: decode -> resize/normalise -> ResNet-50 -> post-process, placed over
    ``world`` GPUs by the balancer (``parallel/placement.py``)."""
    d = definition(batch, graph, height, width, lanes)
    d["name"] = "p_resnet50_pp"
    d["graph"] = ["(SyntheticFrames FrameResize ResNet50Classifier ClassifierTopK)"]
    # resize stays uint8 (224x224x3): cut after it, the stage boundary is 150 KB per frame; the
    # ResNet stage normalises into its stem buffer itself
    # FrameResize writes into frame-held pool slots: the hop sends them without a staging copy
    pre = {"name": "FrameResize", "input": [{"name": "images", "type": "tensor"}],
           "output": [{"name": "images", "type": "tensor"}],
           "parameters": {"image_size": 224, "pool": max(6, 2 * world + 2)},
           "deploy": {"local": {"module": ELEMENTS}}}
    d["elements"].insert(1, pre)
    d["elements"][3]["parameters"]["gather"] = False
    # the frame pool is the pipeline's credit window: two batches in flight per rank
    d["elements"][0]["parameters"]["pool"] = max(6, 2 * world + 2)
    d["parallel"] = {"mode": "pp", "gpus": world}
    return d


def parse_args(argv=None) -> argparse.Namespace:
    """Command line -> options with the per-model defaults applied (batch, frame size)."""
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per GPU per step (default: ResNet-50 640 (both --parallel modes), "
                         "YOLOv8-n 192, Whisper 28 streams).  Batches are sized for the chip's 256 CUs: "
                         "ResNet-50 at B = 320 k runs stage 3 as 245 k tiles of 256 rows (96 %% of the "
                         "CUs busy per round) where B=256 gives 196 tiles (77 %%) and 448 / 768 land "
                         "on 1.34 / 2.3 rounds.  Round-6 sweep, one MI355X, interleaved x 2 "
                         "(scripts/batch_ab_r4.sh): B=320 89.0k (p50 7.7-9.0 ms), 448 86.9-87.6k, 512 "
                         "89.0-90.4k, 640 92.3-92.7k (p50 14 ms), 768 89.5-89.8k, 960 91.3-92.1k, 1280 "
                         "93.2-93.3k (p50 28-31 ms): 640 takes +3.7 %% for 2x the latency.  YOLOv8-n "
                         "(scripts/batch_sweep_r6.sh, probe/yolo_batch_sweep.sh): B=64 44.5-46.4k, 128 "
                         "48.8-48.9k, 192 49.5-50.4k (p50 7.8 ms), 256 50.4k, 320 50.6-51.0k.  "
                         "Whisper-small: 14 streams 3.36-3.38k, 28 3.42k, 42 3.42k windows/s.  Config 3 (--parallel "
                         "pp, world 1): B=320 79.6-79.9k, 640 83.4-84.1k (scripts/probe/pp_batch_ab.sh)")
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
    ap.add_argument("--link-gbps", type=float, default=50.0,
                    help="(pp) xGMI point-to-point rate the balancer prices stage boundaries at")
    ap.add_argument("--parallel", choices=["dp", "pp"], default="dp",
                    help="dp: every GPU runs the whole pipeline (config 2/headline); "
                         "pp: config 3 as balanced multi-GPU actor pipelines (stages + replicas, "
                         "MQTT metadata, RCCL P2P tensors)")
    ap.add_argument("--ingest", choices=["hbm", "host"], default="hbm",
                    help="hbm: frames born in HBM (a hardware decoder); host: frames in pinned host "
                         "memory, uploaded per rank by FrameUpload on a copy stream (PCIe ingest)")
    ap.add_argument("--element-times", default=None,
                    help="(pp) JSON {element: ms per batch} for the stage balancer, or @file")
    ap.add_argument("--write-element-times", default=None,
                    help="(pp) write the measured per-element GPU ms per batch (rank 0's elements, "
                         "its local copy of the replicated stage included) to this file")
    ap.add_argument("--pcie-gbps", type=float, default=50.0,
                    help="(pp, --ingest host) one rank's host->device rate the planner prices "
                         "the upload at (PCIe Gen5 x16 ~50 GB/s)")
    a = ap.parse_args(argv)
    explicit_hw = "--height" in (sys.argv[1:] if argv is None else argv)
    if (a.parallel == "pp" or a.model == "yolov8n") and not explicit_hw:
        a.height, a.width = 480, 640          # configs 3/4 decode VGA video frames
    if a.batch is None:
        a.batch = 192 if a.model == "yolov8n" else 28 if a.model.startswith("whisper") else 640
    return a


def main(argv=None):
    a = parse_args(argv)

    procs = []
    if a.parallel == "pp":
        os.environ.setdefault("AIKO_GPU_TIMING", "1")       # per-stage GPU ms (element events)
        procs = _control_plane(int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")))
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
        return run_pp(a, device, procs)
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
        yd = yolo_definition(a.batch, not a.no_graph, a.height, a.width, a.fanout, a.lanes)
        if a.ingest == "host":          # per-rank ingest: each rank uploads its own batch, no fan-out
            yd = host_ingest(yd)
            yd["parameters"]["spmd"] = False
        d = parse_pipeline_definition_dict(yd)
        result_key, model_cfg = "detections", {"model": "yolov8n", "image_size": [640, 640],
                                               "frame_size": [a.height, a.width], "fanout": a.fanout,
                                               "pipeline": d.graph[0], "gpu_lanes": a.lanes}
        metric = YOLO_METRIC
    else:
        rd = definition(a.batch, not a.no_graph, a.height, a.width, a.lanes)
        if a.ingest == "host":
            rd = host_ingest(rd)
        d = parse_pipeline_definition_dict(rd)
        result_key, model_cfg = "topk", {"model": "resnet50", "image_size": [a.height, a.width],
                                         "pipeline": rd["graph"][0], "gpu_lanes": a.lanes}
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

    # setup (untimed, before the W warmup steps): the first frames tune the conv tiles and capture
    # one hipGraph per frame-pool slot and lane (graphs read the slots in place, no input copy),
    # so even a short warmup starts the timed region in steady state
    for _ in range(SETUP_FRAMES):
        step(False)
    drain(False)
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

    lat = sorted(latencies)
    p99_local = lat[min(len(lat) - 1, int(0.99 * len(lat)))] if lat else 0.0
    t = torch.tensor([elapsed, statistics.median(latencies) if latencies else 0.0, p99_local],
                     dtype=torch.float64, device=device)
    D.all_reduce_max(t)
    elapsed, p50, p99 = float(t[0]), float(t[1]), float(t[2])
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
                     f"synthetic (random uint8 {a.height}x{a.width} frames "
                     + ("in pinned host memory, uploaded per step over PCIe" if a.ingest == "host" else "generated in HBM")
                     + "; random-init weights)"),
            "p50_latency_ms": round(p50 * 1e3, 3),
            "p99_latency_ms": round(p99 * 1e3, 3),
            "config": dict({"global_batch": ws * a.batch, "seq_len": None, "per_gpu_batch": a.batch,
                            "parallelism": f"dp{ws}", "hipgraph": not a.no_graph, "ingest": a.ingest,
                            "setup_frames": SETUP_FRAMES}, **model_cfg),
        }
        if a.model.startswith("whisper"):
            out["audio_seconds_per_s"] = round(ws * a.batch * a.chunk * a.steps / elapsed, 1)
            if a.transcribe:
                out["decoded_tokens_per_s"] = round(ws * a.batch * a.transcribe * a.steps / elapsed, 1)
        print(json.dumps(out), flush=True)
    D.barrier()
    D.destroy()


# per-element GPU ms per frame batch on one MI355X (VGA frames), the balancer's default input:
# the committed measurement (profiles/element_times_r5.json, written by a world-1
# `bench.py --parallel pp --write-element-times` run from each element's HIP events), else
# these round-2 estimates.  Override: --element-times '{"ResNet50Classifier": 3.3, ...}' | @file
PP_ELEMENT_MS = {"SyntheticFrames": 0.01, "FrameResize": 0.06, "ResNet50Classifier": 3.0,
                 "ClassifierTopK": 0.03}
_TIMES_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "element_times_r5.json")


def _load_times(spec):
    """--element-times: inline JSON or @file; a file may hold {"element_ms": {...}}."""
    if not spec:
        return {}
    text = open(spec[1:]).read() if spec.startswith("@") else spec
    d = json.loads(text)
    return {k: float(v) for k, v in d.get("element_ms", d).items()}


if os.path.exists(_TIMES_FILE):
    try:
        PP_ELEMENT_MS = dict(PP_ELEMENT_MS, **_load_times("@" + _TIMES_FILE))
    except (OSError, ValueError):
        pass


def pp_boundary_bytes(batch: int, height: int, width: int) -> dict:
    """Bytes each element hands to the next per frame batch (the hop payload if cut there)."""
    return {"SyntheticFrames": batch * height * width * 3, "FrameUpload": batch * height * width * 3,
            "FrameResize": batch * 224 * 224 * 3,
            "ResNet50Classifier": batch * 1000 * 2, "ClassifierTopK": batch * 5 * 8}


def _control_plane(ws, rank):
    """Config 3 runs as actor pipelines: an MQTT broker and a registrar (subprocesses of rank 0,
    started before anything touches the GPU) carry discovery and per-frame metadata."""
    import subprocess
    port = int(os.environ.get("MASTER_PORT", "29500")) + 7
    os.environ.update({"AIKO_MQTT_HOST": "127.0.0.1", "AIKO_MQTT_PORT": str(port), "AIKO_MQTT_DISABLE": "0",
                       "AIKO_NAMESPACE": f"bench{port}", "AIKO_REGISTRAR_SEARCH_TIMEOUT": "0.5",
                       "AIKO_LOG_MQTT": "false"})
    procs = []
    if rank == 0:
        procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.message.mqtt_broker",
                                       "--host", "127.0.0.1", "--port", str(port)],
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        import socket
        deadline = time.time() + 60
        while True:                            # a fresh box's first python start can take a while
            try:
                socket.create_connection(("127.0.0.1", port), timeout=0.5).close()
                break
            except OSError:
                if time.time() > deadline or procs[0].poll() is not None:
                    raise RuntimeError(f"MQTT broker did not start on port {port}")
                time.sleep(0.1)
        procs.append(subprocess.Popen([sys.executable, "-m", "aiko_services_amd.tools.registrar"],
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
    return procs


def run_pp(a, device, procs):
    """Config 3 as multi-GPU ACTOR pipelines (the path ``aiko_pipeline create`` takes for a
    ``parallel`` definition): the balancer cuts decode -> resize -> ResNet-50 -> post-process
    into stages and replicas (``parallel/placement.py``), every rank runs its stage Pipeline
    registered with the registrar, frames hop between ranks as ``process_frame`` metadata over
    MQTT with the tensors on RCCL P2P (``parallel/hop.py``).  frames/s counted at rank 0 (each
    frame batch is processed once by the whole node)."""
    import threading
    from aiko_services_amd.parallel import dist as D
    from aiko_services_amd.parallel import hop
    from aiko_services_amd.parallel.launch import create_rank_pipeline
    from aiko_services_amd.parallel.placement import make_plan
    from aiko_services_amd.runtime.process import aiko
    ws, rank = D.world_size(), D.rank()
    times = dict(PP_ELEMENT_MS, **_load_times(a.element_times))
    d = pp_definition(a.batch, not a.no_graph, a.height, a.width, ws, a.lanes)
    if a.ingest == "host":
        d = host_ingest(d)
        # where the host frames enter HBM is the planner's call (placement.plan_ingest):
        # per-rank PCIe ingest (SPMD, nothing on xGMI) or rank-0 ingest + a stage cut
        d["parallel"].update(ingest="auto", frame_bytes=a.batch * a.height * a.width * 3,
                             pcie_gbps=a.pcie_gbps)
        times.setdefault("FrameUpload", 0.0)
    from aiko_services_amd.parallel.placement import boundary_ms_from_bytes
    boundary = boundary_ms_from_bytes(pp_boundary_bytes(a.batch, a.height, a.width), a.link_gbps)
    if ws == 1:
        # one GPU: the two-stage actor topology with the ResNet stage as rank 0's local share
        # (exercises the hop-free LocalStage path, frame lanes across the stage boundary)
        order = [e["name"] for e in d["elements"]]
        cut = order.index("ResNet50Classifier")
        plan = make_plan(d, gpus=1, stages=[order[:cut], order[cut:]],
                         replicas=[1, 0], local_share=1.0, group=f"bench{os.environ.get('MASTER_PORT', '0')}")
    else:
        plan = make_plan(d, gpus=ws, times_ms=times, group=f"bench{os.environ.get('MASTER_PORT', '0')}",
                         boundary_ms=boundary)
    plane = hop.init_plane(plan.links, device=device, depth=4)
    responses: queue.Queue = queue.Queue()
    # (per-rank ingest, an SPMD plan: every rank drives and collects its own frames)
    pipeline = create_rank_pipeline(plan, rank, queue_response=responses if rank == 0 or plan.mode == "dp" else None,
                                    grace_time=3600, auto_start=False)
    result = {}

    def driver():
        torch.cuda.set_device(device)
        try:
            result["out"] = _drive_pp(a, pipeline, plane, plan, responses, rank, ws)
        except BaseException as exc:          # report, but still release the other ranks
            result["error"] = repr(exc)
        plane.barrier()                        # rank 0 finished timing: everyone stops
        torch.cuda.synchronize()
        # measured GPU ms per frame of this rank's stage (its elements' events; rank 0 includes
        # its local copy of the replicated stage, weighted by the share of frames it ran)
        mine = pipeline.gpu_element_ms()
        for el in getattr(pipeline, "remote_pipelines", {}).values():
            replicas = el[2]
            for proxy in (replicas.proxies if replicas is not None else []):
                child = getattr(proxy, "pipeline", None)
                if child is not None:
                    share = plan.local_share
                    for k, v in child.gpu_element_ms().items():
                        mine[f"local:{k}"] = round(v * share, 4)
        if plane.control is not None:
            import torch.distributed as tdist
            gathered = [None] * ws
            tdist.all_gather_object(gathered, mine, group=plane.control)
        else:
            gathered = [mine]
        if result.get("out") is not None:
            result["out"]["config"]["measured_rank_ms"] = [round(sum(g.values()), 4) for g in gathered]
            result["out"]["config"]["measured_element_ms"] = gathered
            if a.write_element_times and rank == 0:
                # rank 0's elements (its local copy of the replicated stage at full weight), keyed
                # by the definition's element names; the HIP-event times of one frame overlap the
                # other lane's work, so they are scaled to add up to the measured ms per step —
                # the throughput cost per batch the balancer divides between GPUs
                names = {e["name"].lower(): e["name"] for e in d["elements"]}
                el = {}
                for k, v in gathered[0].items():
                    if k.startswith("local:"):
                        k, v = k[len("local:"):], v / (plan.local_share or 1.0)
                    el.setdefault(names.get(k.lower(), k), v)
                step = result["out"]["ms_per_step"]
                scale = step / max(1e-9, sum(el.values()))
                with open(a.write_element_times, "w") as f:
                    json.dump({"element_ms": {k: round(v * scale, 4) for k, v in el.items()},
                               "raw_event_ms": {k: round(v, 4) for k, v in el.items()},
                               "ms_per_step": step, "batch": a.batch, "frame_size": [a.height, a.width],
                               "lanes": a.lanes,
                               "source": "bench.py --parallel pp --write-element-times (world 1): median "
                                         "HIP-event ms per element and frame batch, scaled to the "
                                         "measured ms per step"}, f, indent=1)
        aiko.process.terminate(0)

    threading.Thread(target=driver, daemon=True, name="bench-driver").start()
    try:
        aiko.process.run(mqtt_connection_required=True)    # event loop on the main thread
    except SystemExit as exc:
        if exc.code:
            result.setdefault("error", f"event loop exit {exc.code} (MQTT broker unreachable?)")
    if result.get("out") is not None:
        print(json.dumps(result["out"]), flush=True)
    for p in procs:
        p.terminate()
    if result.get("error") or (rank == 0 and result.get("out") is None):
        print(f"rank {rank}: {result.get('error', 'no result')}", file=sys.stderr, flush=True)
        os._exit(1)
    os._exit(0)


def _drive_pp(a, pipeline, plane, plan, responses, rank, ws):
    deadline = time.time() + 120
    while pipeline.share.get("lifecycle") != "ready":
        if time.time() > deadline:
            raise RuntimeError(f"rank {rank}: stage pipeline not ready (downstream not discovered)")
        time.sleep(0.02)
    plane.barrier()                            # every stage of the plan is up
    spmd = plan.mode == "dp"                   # per-rank ingest: every rank runs the whole chain
    if rank != 0 and not spmd:
        return None
    from aiko_services_amd.runtime.actor import ActorTopic
    pipeline._post_message(ActorTopic.IN, "create_stream", ["bench", None, {}, 3600, responses, None])
    while "bench" not in pipeline.stream_leases:
        time.sleep(0.01)
    depth = max(a.depth, 2 * ws)
    state = {"frame_id": 0}
    latencies: list = []

    def run(n, record):
        sent = done = 0
        while done < n:
            while sent < n and sent - done < depth:
                # the pipeline's credit window (SyntheticFrames' pool) bounds frames in flight
                if not pipeline.admit_frame("bench", state["frame_id"], timeout=0 if sent > done else 120):
                    break
                pipeline.create_frame({"stream_id": "bench", "frame_id": state["frame_id"]}, {})
                state["frame_id"] += 1
                sent += 1
            info, o = responses.get(timeout=120)
            done += 1
            if info["state"] != 0:
                raise RuntimeError(f"pipeline frame failed: {info} {o}")
            res = o["topk"]
            res.wait()
            if record:
                latencies.append(res.latency)
    run(max(a.warmup, 3 * ws), False)          # every replica tunes + captures its graphs
    torch.cuda.synchronize()
    if spmd:
        plane.barrier()
    t0 = time.perf_counter()
    run(a.steps, True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    frames = a.batch * a.steps
    if spmd and plane.control is not None:
        # every rank ran its own batches: the node's frames over the slowest rank's time
        import torch.distributed as tdist
        got = [None] * ws
        tdist.all_gather_object(got, elapsed, group=plane.control)
        elapsed = max(got)
        frames *= ws
        if rank != 0:
            return None
    p50 = statistics.median(latencies) if latencies else 0.0
    return {
        "metric": METRIC, "value": round(frames / elapsed, 1), "unit": "frames/s", "n_gpus": ws,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "bf16",
        "data": f"synthetic (random uint8 {a.height}x{a.width} frames generated in HBM; random-init weights)",
        "p50_latency_ms": round(p50 * 1e3, 3),
        "config": {"model": "resnet50", "global_batch": a.batch, "seq_len": None,
                   "image_size": [224, 224], "frame_size": [a.height, a.width],
                   "per_gpu_batch": a.batch, "parallelism": f"pp{ws}", "hipgraph": not a.no_graph,
                   "stages": plan.stages, "replicas": plan.replicas, "local_share": round(plan.local_share, 4),
                   "ingest": plan.predicted_ms.get("ingest", "hbm"),
                   "predicted_rank_ms": plan.predicted_ms.get("per_rank_ms"),
                   "transport": "actor pipelines: MQTT metadata + RCCL P2P tensors",
                   "hop": plane.stats(),
                   "hop_bytes_per_frame": round(plane.counters["sent_bytes"] / max(1, plane.counters["sent_msgs"])
                                                / a.batch),
                   "boundary_ms": plan.predicted_ms.get("boundary_ms"),
                   "pipeline": "(SyntheticFrames FrameResize ResNet50Classifier ClassifierTopK)"},
    }


if __name__ == "__main__":
    main()
