"""GPU-resident vision PipelineElements (MI355X): the ResNet-50 pipeline of BASELINE configs 2/3.

    "(SyntheticFrames ResNet50Classifier ClassifierTopK)"                    config 2 / bench
    "(SyntheticFrames ImagePreprocess ResNet50Classifier ClassifierTopK)"    config 3 stages

* ``SyntheticFrames`` — the "decode" stage: a batch of ``batch`` uint8 RGB frames of
  ``height`` x ``width`` produced directly in HBM (a rotating pool of ``pool`` random batches,
  like a hardware decoder writing into device memory; no host upload on the hot path).  In a
  stream it can also run as a frame generator (``frames``, ``rate``).  With ``global: true``
  only rank ``src`` produces frames — ``world x batch`` of them — for a FrameFanout.
* ``FrameUpload`` — host frames (a decoder / camera / file reader in host memory, or
  ``SyntheticFrames`` with ``host: true``) -> a FramePool slot in HBM: pinned staging, the
  H2D copy on the element's own copy stream (it overlaps the previous frames' compute), the
  frame's lane ordered after it by an event, the slot held until the frame completes.
* ``ImagePreprocess`` — fused bilinear resize + ImageNet normalise + NHWC->padded-4-channel
  layout in one HIP kernel (output: the ResNet stem buffer).
* ``ResNet50Classifier`` — ResNet-50 on the igemm MFMA kernels; accepts uint8 frames (then
  pre-processes itself) or a stem buffer; emits logits; optional hipGraph capture.
* ``ClassifierTopK`` — softmax + top-k kernel; with data parallelism (torch.distributed over
  RCCL) all-gathers the results to every rank; copies them to pinned host memory without
  synchronising and emits a :class:`DeviceResult`.
"""
from __future__ import annotations

import time

import torch

from ...gpu.element import DeviceResult, FramePool, GpuPipelineElement, HostRing
from ...pipeline.stream import StreamEvent

__all__ = ["SyntheticFrames", "FrameUpload", "FrameResize", "ImagePreprocess", "ResNet50Classifier",
           "ClassifierTopK"]


def _int(v, d):
    try:
        return int(v)
    except (TypeError, ValueError):
        return d


class SyntheticFrames(GpuPipelineElement):
    """The "decode" stage: frame batches written into slots of an HBM :class:`FramePool` (each
    slot filled once with random pixels, like a hardware decoder writing device memory).  Every
    frame holds its slot until the frame completes and the GPU is done with it; with all
    ``pool`` slots in flight the next frame waits for the oldest (back-pressure on the device
    queue, at most ``acquire_timeout`` s) or — ``on_exhausted: drop`` — is dropped (DROP_FRAME).
    The pool size is also the pipeline's credit window for generated frames
    (``PipelineImpl.limit_frames``).  Stable slot addresses let
    the downstream hipGraphs be captured on the slots themselves (no input copy)."""
    lane_safe = True          # read-only frame pool

    def __init__(self, context):
        context.set_protocol("synthetic_frames:0")
        super().__init__(context)
        self.frame_pool = None
        self._shape = None
        self.dropped = 0
        # ``stamp: true`` (tests): the frame id goes into the first 8 bytes of its slot, so a
        # frame's pixels — and every output computed from them — depend on the frame id alone,
        # not on which slot it was served from
        self._stamp = str(self.get_parameter("stamp", False)[0]).lower() in ("true", "1", "yes")

    def _ensure_pool(self, glob):
        if self.frame_pool is not None:
            return
        from ...gpu.element import FramePool
        B = _int(self.get_parameter("batch", 1)[0], 1)
        if self.pipeline is not None and hasattr(self.pipeline, "limit_frames"):
            # generated frames in flight never exceed the slots (the generator thread waits
            # for a credit): the actor thread's acquire below then never waits for a slot that
            # only a later message on the same thread could free
            self.pipeline.limit_frames(self.name, max(1, _int(self.get_parameter("pool", 2)[0], 2)))
        if glob:
            from ...parallel import dist as D
            B *= D.world_size()
        H = _int(self.get_parameter("height", 224)[0], 224)
        W = _int(self.get_parameter("width", 224)[0], 224)
        n = max(1, _int(self.get_parameter("pool", 2)[0], 2))
        seed = _int(self.get_parameter("seed", 0)[0], 0)
        self._shape = (B, H, W, 3)
        self.frame_pool = FramePool(n, B * H * W * 3, device=self.device)
        g = torch.Generator(device=self.device).manual_seed(seed)
        slots = [self.frame_pool.acquire(0) for _ in range(n)]
        same = None
        if self._stamp:                       # every slot the same pixels: only the stamp differs
            same = torch.randint(0, 256, self._shape, dtype=torch.uint8, device=self.device, generator=g)
        for s in slots:
            v = self.frame_pool.view(s, self._shape, torch.uint8)
            v.copy_(same if same is not None else
                    torch.randint(0, 256, self._shape, dtype=torch.uint8, device=self.device, generator=g))
        for s in slots:
            self.frame_pool.release_after(s)

    def _host_frames(self):
        """``host: true`` — the decoder's output in pinned HOST memory (``pool`` pre-filled
        batches served in rotation, read-only), for a FrameUpload to bring into HBM."""
        if getattr(self, "host_pool", None) is None:
            B = _int(self.get_parameter("batch", 1)[0], 1)
            H = _int(self.get_parameter("height", 224)[0], 224)
            W = _int(self.get_parameter("width", 224)[0], 224)
            n = max(1, _int(self.get_parameter("pool", 2)[0], 2))
            g = torch.Generator().manual_seed(_int(self.get_parameter("seed", 0)[0], 0))
            pin = torch.cuda.is_available()
            self.host_pool = [torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g).pin_memory()
                               if pin else torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, generator=g)
                               for _ in range(n)]
            self._next = 0
        frames = self.host_pool[self._next]
        self._next = (self._next + 1) % len(self.host_pool)
        return frames

    def _frames(self, stream=None):
        if str(self.get_parameter("host", False)[0]).lower() in ("true", "1", "yes"):
            return self._host_frames()
        glob = str(self.get_parameter("global", False)[0]).lower() in ("true", "1", "yes") \
            and str(self.get_parameter("spmd", True)[0]).lower() not in ("false", "0", "no")
        if glob:
            # data-parallel ingest: rank ``src`` decodes the node's whole batch (N x batch),
            # the other ranks get theirs from FrameFanout
            from ...parallel import dist as D
            if D.rank() != _int(self.get_parameter("src", 0)[0], 0):
                return None
        self._ensure_pool(glob)
        drop = str(self.get_parameter("on_exhausted", "block")[0]).lower() == "drop"
        # "block" waits for the GPU to finish the oldest frame, bounded: frames pushed in past the
        # credit window (direct process_frame calls) are dropped rather than wedging the actor
        timeout = self.get_parameter("acquire_timeout", 30.0)[0]
        slot = self.frame_pool.acquire(0.0 if drop else float(timeout))
        if slot < 0:
            return False
        self.hold_for_frame(self.frame_pool, slot)
        from ...parallel.hop import mark_frame_held
        v = self.frame_pool.view(slot, self._shape, torch.uint8)
        if self._stamp:
            stamp = torch.tensor([int(getattr(stream, "frame_id", 0) or 0)], dtype=torch.int64).view(torch.uint8)
            v.view(-1)[:8].copy_(stamp.to(self.device, non_blocking=False))
        # the slot is the frame's until it completes: a hop may send it zero-copy
        return mark_frame_held(v)

    def start_stream(self, stream, stream_id):
        limit, found = self.get_parameter("frames")
        if found and limit:
            if self.pipeline is not None and hasattr(self.pipeline, "limit_frames"):
                # the credit window must be known before the generator admits its first frame
                # (the pool itself is made on the first frame): else a burst of admitted frames
                # waits on the actor thread for slots only their own responses could free
                self.pipeline.limit_frames(self.name, max(1, _int(self.get_parameter("pool", 2)[0], 2)))
            stream.variables["synthetic_left"] = int(limit)
            rate, _ = self.get_parameter("rate", None)
            self.create_frames(stream, self.frame_generator, rate=float(rate) if rate else None)
        return StreamEvent.OKAY, None

    def frame_generator(self, stream, frame_id):
        left = stream.variables.get("synthetic_left", 0)
        if left <= 0:
            return StreamEvent.STOP, {"diagnostic": "All frames generated"}
        stream.variables["synthetic_left"] = left - 1
        return StreamEvent.OKAY, {"t_submit": time.perf_counter()}

    def process_frame(self, stream, **kwargs):
        frames = self._frames(stream)
        if frames is False:
            self.dropped += 1
            self.share["frames_dropped"] = self.dropped
            return StreamEvent.DROP_FRAME, {"diagnostic": "frame pool exhausted"}
        return StreamEvent.OKAY, {"images": frames, "t_submit": kwargs.get("t_submit", time.perf_counter())}


class FrameUpload(GpuPipelineElement):
    """Host -> HBM ingest of a frame batch (SURVEY K11 "synthetic-frame source + upload"; the
    reference decodes into host memory and hands numpy images on,
    ``/root/reference/src/aiko_services/elements/media/video_io.py:124-166``,
    ``image_io.py:180-191``).

    ``images``: a host uint8 tensor [B, H, W, 3] (pinned or pageable), one HxWx3 image, or a
    list of them (numpy arrays from ``VideoReadFile`` / ``ImageReadFile`` / ``VideoReadWebcam``).
    Pageable input is first copied into a pinned staging set (a ring of ``staging`` sets, each
    reused once its previous upload finished).  The H2D copy runs on this element's copy
    stream into a FramePool slot (``pool`` slots of the batch's size), the frame's lane waits
    on the copy's event, and the slot is held until the frame completes — so the upload of
    frame k+1 overlaps the compute of frame k, and a hop can send the slot zero-copy
    (``mark_frame_held``).  Output ``images``: the device batch, uint8 [B, H, W, 3]."""
    lane_safe = True

    def __init__(self, context):
        context.set_protocol("frame_upload:0")
        super().__init__(context)
        pool, explicit = self.get_parameter("pool", 6)
        self.pool_slots = max(2, _int(pool, 6))
        self.pool_explicit = bool(explicit)
        self.staging_sets = max(2, _int(self.get_parameter("staging", 4)[0], 4))
        self._pools = {}
        self._staging = {}
        self._copy_stream = torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None
        self.bytes_uploaded = 0

    @staticmethod
    def _as_batch(images):
        import numpy as np
        if isinstance(images, torch.Tensor):
            return images if images.dim() == 4 else images.unsqueeze(0)
        if isinstance(images, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(images))
            return t if t.dim() == 4 else t.unsqueeze(0)
        if isinstance(images, (list, tuple)) and images:
            return [torch.from_numpy(np.ascontiguousarray(i)) if isinstance(i, np.ndarray) else i for i in images]
        raise ValueError("FrameUpload: images must be a uint8 tensor / array [B, H, W, 3] or a list of HxWx3")

    def _pinned(self, batch, shape):
        """A pinned host set holding ``batch`` (a tensor or a list of images)."""
        if isinstance(batch, torch.Tensor) and (batch.is_pinned() or self.device.type != "cuda"):
            return batch.contiguous()
        ring = self._staging.get(shape)
        if ring is None:
            ring = self._staging[shape] = {"sets": [torch.empty(shape, dtype=torch.uint8, pin_memory=True)
                                                    for _ in range(self.staging_sets)],
                                           "events": [None] * self.staging_sets, "next": 0}
        i = ring["next"]
        ring["next"] = (i + 1) % self.staging_sets
        ev = ring["events"][i]
        if ev is not None:
            ev.synchronize()                      # its upload (staging_sets frames ago) is done
        host = ring["sets"][i]
        if isinstance(batch, torch.Tensor):
            host.copy_(batch)
        else:
            for j, img in enumerate(batch):
                host[j].copy_(img)
        ring["current"] = i
        return host

    def _credit_window(self) -> int:
        """Frames a replicated / remote plan keeps in flight: 2 x hop depth x hop_batch x
        members (the engine's default frame window), 0 without remote elements."""
        pl = self.pipeline
        if pl is None or not getattr(pl, "remote_pipelines", None):
            return 0
        from ...parallel import hop as _hop
        hop = _hop.plane()
        depth = hop.depth if hop is not None else 4
        return 2 * depth * pl.hop_batch * max(1, pl._remote_member_count())

    def _size_pool(self):
        # without an explicit ``pool`` the slots follow the plan's credit window, so a rank-0
        # ingest feeding k replicas keeps every replica busy (6 slots capped them all)
        if not self.pool_explicit:
            self.pool_slots = max(self.pool_slots, self._credit_window())
        if self.pipeline is not None and hasattr(self.pipeline, "limit_frames"):
            self.pipeline.limit_frames(self.name, self.pool_slots)

    def start_stream(self, stream, stream_id):
        # each frame holds one upload slot until it completes (longer when a hop sends the slot
        # zero-copy): the pipeline's frame window must not exceed the slots, or the actor would
        # wait in acquire() for a slot only a later response on this same thread frees
        self._size_pool()
        return StreamEvent.OKAY, None

    def process_frame(self, stream, images):
        from ...parallel.hop import mark_frame_held
        batch = self._as_batch(images)
        first = batch if isinstance(batch, torch.Tensor) else batch[0]
        shape = (len(batch),) + tuple(first.shape[-3:]) if not isinstance(batch, torch.Tensor) else tuple(batch.shape)
        if len(shape) != 4 or shape[3] != 3:
            raise ValueError(f"FrameUpload: expected [B, H, W, 3] frames, got {shape}")
        if self.device.type != "cuda":
            out = batch if isinstance(batch, torch.Tensor) else torch.stack(batch)
            return StreamEvent.OKAY, {"images": out.to(torch.uint8)}
        nbytes = shape[0] * shape[1] * shape[2] * 3
        pool = self._pools.get(shape)
        if pool is None:
            self._size_pool()                     # the plan's members are discovered by now
            pool = self._pools[shape] = FramePool(self.pool_slots, nbytes, device=self.device)
        slot = pool.acquire(30.0)
        if slot < 0:
            return StreamEvent.DROP_FRAME, {"diagnostic": "upload pool exhausted"}
        host = self._pinned(batch, shape)
        dst = pool.view(slot, shape, torch.uint8)
        cur = torch.cuda.current_stream(self.device)
        ev = torch.cuda.Event()
        with torch.cuda.stream(self._copy_stream):
            dst.copy_(host, non_blocking=True)
            ev.record(self._copy_stream)
        cur.wait_event(ev)                        # the frame's next kernels follow the upload
        ring = self._staging.get(shape)
        if ring is not None and host is ring["sets"][ring.get("current", 0)]:
            ring["events"][ring["current"]] = ev  # the staging set is free once this copy is
        self.hold_for_frame(pool, slot)
        self.bytes_uploaded += nbytes
        self.share["bytes_uploaded"] = self.bytes_uploaded
        return StreamEvent.OKAY, {"images": mark_frame_held(dst)}


class FrameResize(GpuPipelineElement):
    """The "resize" stage of config 3: bilinear uint8 -> uint8 resize of a frame batch to
    ``image_size`` (square) on the GPU.  Placed before a stage cut it makes the boundary the
    small uint8 frame (150 KB per 224² frame) instead of the normalised bf16 stem buffer
    (427 KB): ResNet50Classifier accepts uint8 frames and pre-processes them itself."""
    lane_safe = True

    def __init__(self, context):
        context.set_protocol("frame_resize:0")
        super().__init__(context)
        self.size = _int(self.get_parameter("image_size", 224)[0], 224)
        # ``pool: N`` — resize into N FramePool slots, each held by its frame until the frame
        # completes: before a stage cut the hop then sends the slot itself (no staging copy,
        # ``parallel/hop.py`` mark_frame_held); 0 = one buffer per lane, reused every frame
        self.pool_slots = _int(self.get_parameter("pool", 0)[0], 0)
        self._out = {}
        self._pools = {}

    def process_frame(self, stream, images):
        from ...ops import vision as V
        B = images.shape[0]
        if images.shape[1] == self.size and images.shape[2] == self.size:
            return StreamEvent.OKAY, {"images": images}
        shape = (B, self.size, self.size, 3)
        if self.pool_slots > 0:
            pool = self._pools.get(B)
            if pool is None:
                pool = self._pools[B] = FramePool(self.pool_slots, B * self.size * self.size * 3, device=self.device)
            slot = pool.acquire(30.0)
            if slot >= 0:
                out = pool.view(slot, shape, torch.uint8)
                self.hold_for_frame(pool, slot)
                from ...parallel.hop import mark_frame_held
                return StreamEvent.OKAY, {"images": mark_frame_held(V.resize_u8(images, shape[1:3], out=out))}
        out = self._out.get((B, self.lane))
        if out is None:
            out = self._out[(B, self.lane)] = torch.empty(shape, dtype=torch.uint8, device=self.device)
        return StreamEvent.OKAY, {"images": V.resize_u8(images, (self.size, self.size), out=out)}


class ImagePreprocess(GpuPipelineElement):
    lane_safe = True

    def __init__(self, context):
        context.set_protocol("image_preprocess:0")
        super().__init__(context)
        self.size = _int(self.get_parameter("image_size", 224)[0], 224)
        self._out = {}

    def process_frame(self, stream, images):
        from ...ops import conv as C
        from ...ops import vision as V
        B = images.shape[0]
        Hp, Wp = C.stem_geometry(self.size, self.size)
        out = self._out.get((B, self.lane))
        if out is None:
            out = self._out[(B, self.lane)] = torch.empty(B, Hp, Wp, 4, dtype=torch.bfloat16, device=self.device)
        return StreamEvent.OKAY, {"images": V.preprocess_frames(images, (self.size, self.size), out=out)}


class ResNet50Classifier(GpuPipelineElement):
    lane_safe = True          # one model workspace per lane (buffer tag)

    def __init__(self, context):
        context.set_protocol("resnet50:0")
        super().__init__(context)
        from ...models.resnet50 import ResNet50
        from ...ops import require_native
        require_native()
        seed = _int(self.get_parameter("seed", 0)[0], 0)
        self.model = ResNet50(seed=seed, device=self.device,
                              image_size=_int(self.get_parameter("image_size", 224)[0], 224))
        self.load_model_weights(self.model)
        tune, _ = self.get_parameter("autotune", default=self.gpu_config.autotune)
        self.autotune = str(tune).lower() in ("true", "1", "yes")
        self._tuned = set()
        gate, _ = self.get_parameter("phase_gate", default=__import__("os").environ.get("AIKO_PHASE_GATE", "0"))
        self.phase_gate = str(gate).lower() in ("true", "1", "yes")
        self._gate = None

    def _run(self, images):
        tag = f"lane{self.lane}." if self.lane else ""
        if images.dtype == torch.uint8:
            return self.model.logits(images, tag)       # uint8 fused stem when the size fits
        return self.model.logits_from_stem(images, tag)

    def _run_a(self, images):
        return self.model.logits_part_a(images, f"lane{self.lane}." if self.lane else "")

    def _run_b(self, x):
        return self.model.logits_part_b(x, f"lane{self.lane}." if self.lane else "")

    def process_frame(self, stream, images):
        key = (tuple(images.shape), images.dtype)
        if key not in self._tuned:
            # first frame of a new shape: pick each conv's tile by measurement, then capture
            from ...ops import conv as C
            if self.autotune:
                with C.autotune():
                    self._run(images)
            self._tuned.add(key)
        lanes = getattr(self.pipeline, "_lanes_cfg", (1, None))[0] if self.pipeline is not None else 1
        if self.phase_gate and lanes > 1 and self.device.type == "cuda":
            # lane phase gating (opt-in, ``phase_gate`` / AIKO_PHASE_GATE): this frame's memory-
            # bound half (stem, stages 1-2) starts only once the previous frame (other lane) has
            # finished its own, so it runs beside that frame's compute-bound half.  Measured on
            # one MI355X at B=256: 73.1k vs 73.9k frames/s free-running — the free-running lanes
            # already interleave well, so it stays off by default
            if self._gate is not None:
                torch.cuda.current_stream(self.device).wait_event(self._gate)
            mid = self.run_maybe_captured(("a",) + key, self._run_a, images)
            self._gate = torch.cuda.Event()
            self._gate.record()
            logits = self.run_maybe_captured(("b",) + key, self._run_b, mid)
        else:
            logits = self.run_maybe_captured(key, self._run, images)
        return StreamEvent.OKAY, {"logits": logits}


class ClassifierTopK(GpuPipelineElement):
    lane_safe = True          # device buffers and pinned host ring per lane

    def __init__(self, context):
        context.set_protocol("classifier_topk:0")
        super().__init__(context)
        self.k = _int(self.get_parameter("k", 5)[0], 5)
        gather, _ = self.get_parameter("gather", default=True)
        self.gather = str(gather).lower() in ("true", "1", "yes")
        self._bufs = {}

    @staticmethod
    def _split(flat, rows, k):
        """(prob fp32 [rows, k], index int32 [rows, k]) as contiguous views of one int32 buffer,
        so the per-step device->host result copy is a single transfer."""
        n = rows * k
        return flat[:n].view(torch.float32).view(rows, k), flat[n:].view(rows, k)

    def _buffers(self, B, world):
        key = (B, world, self.lane)
        b = self._bufs.get(key)
        if b is None:
            dev, k = self.device, self.k
            pin = dev.type == "cuda"
            b = {"dev": torch.empty(2 * B * k, dtype=torch.int32, device=dev),
                 "all": torch.empty(2 * world * B * k, dtype=torch.int32, device=dev),
                 "host": HostRing(lambda: torch.empty(2 * world * B * k, dtype=torch.int32,
                                                      pin_memory=pin), 8)}
            self._bufs[key] = b
        return b

    def process_frame(self, stream, logits, t_submit=None):
        from ...ops import vision as V
        from ...parallel import dist as D
        B = logits.shape[0]
        world = D.world_size() if self.gather else 1
        b = self._buffers(B, world)
        prob, index = self._split(b["dev"], B, self.k)
        V.softmax_topk(logits, self.k, prob=prob, index=index)
        flat = b["dev"]
        if world > 1:
            all_prob, all_index = self._split(b["all"], world * B, self.k)
            D.all_gather_into(all_prob, prob)
            D.all_gather_into(all_index, index)
            flat = b["all"]
        frame = self.pipeline.current_frame() if self.pipeline is not None else None
        if getattr(frame, "hop_reply", None) is not None:
            # this stage answers a remote hop: the result goes back as DEVICE tensors (the hop
            # packs them on this stream); the requester decides whether it needs them on the host
            hp, hi = self._split(flat, world * B, self.k)
            ev = None
            if self.device.type == "cuda":
                ev = torch.cuda.Event()
                ev.record()
            return StreamEvent.OKAY, {"topk": DeviceResult(
                {"top_prob": hp, "top_index": hi}, ev,
                t_submit=t_submit if isinstance(t_submit, (float, torch.Tensor)) else None)}
        slot, host = b["host"].acquire()
        host.copy_(flat, non_blocking=True)
        hp, hi = self._split(host, world * B, self.k)
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        result = DeviceResult({"top_prob": hp, "top_index": hi}, ev,
                              t_submit=t_submit if isinstance(t_submit, (float, torch.Tensor)) else None)
        return StreamEvent.OKAY, {"topk": b["host"].bind(slot, result)}
