"""GPU detection PipelineElements — BASELINE config 4, data-parallel YOLOv8 over RCCL.

    "(SyntheticFrames FrameFanout YoloDetector DetectionsGather)"

One process per GPU runs the same pipeline (``torchrun``).  The ingest rank decodes the whole
node's frame batch (``SyntheticFrames`` with ``global: true``); ``FrameFanout`` hands every rank
its share over RCCL — ``scatter`` (grouped point-to-point sends, one per xGMI link: each link
carries 1/N of the batch) or ``broadcast`` (every rank receives the whole batch and keeps its
slice, the reference topology of the BASELINE config);  ``YoloDetector`` runs letterbox +
YOLOv8 + DFL decode + fused top-k/NMS, hipGraph-captured, producing fixed-size detections
``[B, max_det, 6]`` + counts;  ``DetectionsGather`` all-gathers them over RCCL (fixed size, so
no size exchange) into pinned host memory and emits a :class:`DeviceResult` without
synchronising.  (Reference ``examples/yolo/yolo.py:46-87`` ran Ultralytics on one frame at a
time on whatever device it found.)
"""
from __future__ import annotations

import torch

from ...gpu.element import DeviceResult, GpuPipelineElement, HostRing
from ...pipeline.stream import StreamEvent

__all__ = ["FrameFanout", "YoloDetector", "DetectionsGather"]


def _int(v, d):
    try:
        return int(v)
    except (TypeError, ValueError):
        return d


def spmd(element) -> bool:
    """Whether the element's pipeline runs SPMD (``parallel: {mode: dp}``): its collectives
    pair up across ranks.  A replicated-stage plan of the same definition
    (``parallel: {mode: dp, replicated: true}``, ``parallel/placement.py``) sets the pipeline
    parameter ``spmd`` false: every frame then visits ONE replica, so fan-out / gather are
    pass-throughs."""
    return str(element.get_parameter("spmd", True)[0]).lower() not in ("false", "0", "no")


def _bool(v):
    return str(v).lower() in ("true", "1", "yes")


class FrameFanout(GpuPipelineElement):
    lane_safe = True
    """Ingest rank's ``[N*B, H, W, 3]`` batch -> this rank's ``[B, H, W, 3]`` (RCCL)."""

    def __init__(self, context):
        context.set_protocol("frame_fanout:0")
        super().__init__(context)
        self.mode = str(self.get_parameter("mode", "scatter")[0])
        if self.mode not in ("scatter", "broadcast"):
            raise ValueError(f"FrameFanout mode must be scatter|broadcast, not {self.mode}")
        self.src = _int(self.get_parameter("src", 0)[0], 0)
        self._bufs = {}

    def process_frame(self, stream, images=None):
        from ...parallel import dist as D
        ws, rank = D.world_size(), D.rank()
        if ws == 1 or not spmd(self):
            return StreamEvent.OKAY, {"images": images}
        B = _int(self.get_parameter("batch", 1)[0], 1)
        H = _int(self.get_parameter("height", 480)[0], 480)
        W = _int(self.get_parameter("width", 640)[0], 640)
        if rank == self.src:
            if images is None or images.shape[0] != ws * B:
                raise ValueError(f"FrameFanout: ingest rank needs [{ws * B}, H, W, 3] frames")
            H, W = images.shape[1:3]
        if self.mode == "broadcast":
            full = images if rank == self.src else self._buf("full", (ws * B, H, W, 3))
            D.broadcast(full, self.src)
            return StreamEvent.OKAY, {"images": full[rank * B:(rank + 1) * B]}
        mine = self._buf("mine", (B, H, W, 3))
        D.scatter_frames(images if rank == self.src else None, mine, self.src)
        return StreamEvent.OKAY, {"images": mine}

    def _buf(self, key, shape):
        """Receive buffer of this frame: a slot of a per-shape HBM FramePool, held until the
        frame completes (stable addresses: the detector's graphs capture on the slots)."""
        from ...gpu.element import FramePool
        k = (key, shape)
        pool = self._bufs.get(k)
        if pool is None:
            n = shape[0] * shape[1] * shape[2] * shape[3]
            pool = self._bufs[k] = FramePool(_int(self.get_parameter("pool", 4)[0], 4), n, device=self.device)
            self.frame_pool = pool
        slot = pool.acquire()
        self.hold_for_frame(pool, slot)
        return pool.view(slot, shape, torch.uint8)


class YoloDetector(GpuPipelineElement):
    """uint8 RGB frames -> YOLOv8 detections (fixed-size rows + counts), on the HIP kernels."""
    lane_safe = True          # one model workspace per lane

    def __init__(self, context):
        context.set_protocol("yolo_detector:0")
        super().__init__(context)
        from ...models.yolov8 import YOLOv8
        from ...ops import require_native
        require_native()
        p = lambda name, d: self.get_parameter(name, d)[0]  # noqa: E731
        self.model = YOLOv8(scale=str(p("scale", "n")), num_classes=_int(p("classes", 80), 80),
                            seed=_int(p("seed", 0), 0), device=self.device,
                            image_size=_int(p("image_size", 640), 640),
                            conf=float(p("conf", 0.25)), iou=float(p("iou", 0.7)),
                            max_det=_int(p("max_det", 300), 300),
                            max_candidates=_int(p("max_candidates", 1024), 1024))
        self.load_model_weights(self.model)
        self.autotune = _bool(p("autotune", self.gpu_config.autotune))
        self._tuned = set()

    def _run(self, images):
        self.model.ws_tag = f"lane{self.lane}." if self.lane else ""
        return self.model.detect(images)

    def process_frame(self, stream, images):
        key = (tuple(images.shape), images.dtype)
        if key not in self._tuned:
            from ...ops import conv as C
            if self.autotune:
                with C.autotune():
                    self._run(images)
            self._tuned.add(key)
        det, count = self.run_maybe_captured(key, self._run, images)
        return StreamEvent.OKAY, {"detections": det, "counts": count}


class DetectionsGather(GpuPipelineElement):
    """All-gather fixed-size detections over RCCL, copy to pinned host, emit a DeviceResult."""
    lane_safe = True

    def __init__(self, context):
        context.set_protocol("detections_gather:0")
        super().__init__(context)
        self.gather = _bool(self.get_parameter("gather", True)[0])
        self._bufs = {}

    def _buffers(self, shape, world):
        key = (shape, world, self.lane)
        b = self._bufs.get(key)
        if b is None:
            B, D_, six = shape
            dev = self.device
            pin = dev.type == "cuda"
            b = {"all_det": torch.empty(world * B, D_, six, dtype=torch.float32, device=dev),
                 "all_count": torch.empty(world * B, dtype=torch.int32, device=dev),
                 "host": HostRing(lambda: (
                     torch.empty(world * B, D_, six, dtype=torch.float32, pin_memory=pin),
                     torch.empty(world * B, dtype=torch.int32, pin_memory=pin)), 8)}
            self._bufs[key] = b
        return b

    def process_frame(self, stream, detections, counts, t_submit=None):
        from ...parallel import dist as D
        world = D.world_size() if self.gather and spmd(self) else 1
        b = self._buffers(tuple(detections.shape), world)
        det, cnt = detections, counts
        if world > 1:
            D.all_gather_into(b["all_det"], detections)
            D.all_gather_into(b["all_count"], counts)
            det, cnt = b["all_det"], b["all_count"]
        slot, (hd, hc) = b["host"].acquire()
        hd.copy_(det, non_blocking=True)
        hc.copy_(cnt, non_blocking=True)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        result = DeviceResult({"det": hd, "count": hc}, ev,
                              t_submit=t_submit if isinstance(t_submit, (float, torch.Tensor)) else None)
        return StreamEvent.OKAY, {"detections": b["host"].bind(slot, result)}
