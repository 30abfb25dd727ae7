"""GPU-resident PipelineElements and frame-buffer pools.

``GpuPipelineElement`` is a PipelineElement bound to one MI355X (its ``deploy.local.device``,
else this process's GPU) that launches HIP work asynchronously on the current stream and
hands device tensors to its successors through the frame ``swag`` (no copies, no
serialisation).  Optional hipGraph capture (parameter ``graph: true``) replays the element's
whole launch sequence per input shape, removing per-kernel launch cost; inputs are copied
into the captured static buffers when their address differs.

``DeviceResult`` is what a GPU pipeline emits at its output: device/pinned-host tensors plus
the HIP event that completes them — the consumer calls ``wait()`` (or ``ready()``) instead of
the pipeline synchronising the device per frame.

``FramePool`` wraps the native HBM slab pool (``csrc/runtime/frame_pool.cpp``).
"""
from __future__ import annotations

import time
import weakref
from collections import deque

import torch

from ..pipeline.engine import PipelineElement
from ..pipeline.stream import StreamEvent
from ..utils.configuration import get_gpu_configuration
from .device import parse_device, require_gpu

__all__ = ["GpuPipelineElement", "DeviceResult", "FramePool", "CapturedCall", "HostRing"]

# Device addresses known to be reused frame after frame: FramePool slot bases and the static
# outputs of captured graphs.  run_maybe_captured captures a per-address graph at once for
# inputs at these addresses; any other address must recur before it gets one.
_STABLE_PTRS: set = set()
# AIKO_GRAPH_ADMIT=0: every new address gets its own graph at once (round-2 behaviour, A/B)
_ADMIT_ALL = __import__("os").environ.get("AIKO_GRAPH_ADMIT", "1") == "0"

_DTYPE_CODES = {torch.uint8: 0, torch.int8: 1, torch.int16: 2, torch.int32: 3, torch.int64: 4,
                torch.float16: 5, torch.float32: 6, torch.float64: 7, torch.bool: 11,
                torch.bfloat16: 15}


class FramePool:
    """Fixed-size HBM slots with blocking acquire (back-pressure) — native implementation.

    ``release_after(slot)`` is the GPU-aware release: the slot returns to the pool once the
    work queued so far on the current stream has finished (a HIP event, polled on the next
    ``acquire``), so a frame's buffers are recycled only after its kernels stopped reading
    them.  ``acquire(timeout)`` first retires completed releases, then — while releases are
    still pending on the GPU — waits for the oldest one (back-pressure on the device queue)
    before falling back to the native blocking wait; -1 on timeout."""

    def __init__(self, num_slots: int, slot_bytes: int, device=None):
        from ..ops import require_native
        require_native()
        dev = parse_device(device) if device is not None and str(device) != "cpu" else None
        self.device = dev if dev is not None else torch.device("cpu")
        self._pool = torch.classes.aiko.FramePool(int(num_slots), int(slot_bytes),
                                                  dev.index if dev is not None and dev.type == "cuda" else -1)
        self._pending = deque()         # (event | None, slot)
        self._slot_ptrs = [self.view(s, (1,)).data_ptr() for s in range(self.capacity)]
        _STABLE_PTRS.update(self._slot_ptrs)

    def _reap(self, block: bool = False) -> None:
        while self._pending:
            ev, slot = self._pending[0]
            if ev is not None and not ev.query():
                if not block:
                    return
                ev.synchronize()
                block = False
            self._pending.popleft()
            self._pool.release(int(slot))

    def acquire(self, timeout: float | None = None) -> int:
        self._reap()
        if self._pending and self._pool.free_count() == 0:
            self._reap(block=True)          # wait for the GPU to finish the oldest holder
        return self._pool.acquire(-1 if timeout is None else int(timeout * 1000))

    def release(self, slot: int) -> None:
        self._pool.release(int(slot))

    def release_after(self, slot: int) -> None:
        ev = None
        if self.device.type == "cuda":
            ev = torch.cuda.Event()
            ev.record()
        self._pending.append((ev, int(slot)))

    def view(self, slot: int, shape, dtype=torch.uint8) -> torch.Tensor:
        return self._pool.view(int(slot), list(shape), _DTYPE_CODES[dtype])

    def close(self):
        _STABLE_PTRS.difference_update(self._slot_ptrs)
        self._pool.close()

    @property
    def capacity(self):
        return self._pool.capacity()

    @property
    def slot_bytes(self):
        return self._pool.slot_bytes()

    def free_count(self):
        return self._pool.free_count()

    def unheld_count(self) -> int:
        """Slots no frame holds: free ones plus releases still waiting on their GPU event."""
        return self._pool.free_count() + len(self._pending)

    def stats(self) -> dict:
        cap, used, hw, acq, exh = self._pool.stats()
        return {"capacity": cap, "in_use": used, "high_water": hw, "acquired": acq, "exhausted": exh}


class DeviceResult:
    """Tensors produced asynchronously on the GPU plus the event that completes them."""

    __slots__ = ("tensors", "event", "t_submit", "t_done", "meta", "__weakref__")
    __aiko_device_result__ = True       # message/tensor_payload.py: sent as its tensors, re-wrapped

    def __init__(self, tensors: dict, event: torch.cuda.Event | None, t_submit: float | None = None, meta=None):
        self.tensors = tensors
        self.event = event
        self.t_submit = t_submit if t_submit is not None else time.perf_counter()
        self.t_done = None
        self.meta = meta or {}

    def ready(self) -> bool:
        return self.event is None or self.event.query()

    def wait(self) -> dict:
        if self.event is not None:
            self.event.synchronize()
        if self.t_done is None:
            self.t_done = time.perf_counter()
        return self.tensors

    @property
    def latency(self):
        if self.t_done is None:
            return None
        t = self.t_submit
        if isinstance(t, torch.Tensor):      # int64 ns stamp carried through a PP stage header
            t = int(t.reshape(-1)[0]) * 1e-9
        return self.t_done - t

    def __repr__(self):
        shapes = {k: tuple(v.shape) if hasattr(v, "shape") else v for k, v in self.tensors.items()}
        return f"DeviceResult({shapes}, ready={self.ready()})"


class HostRing:
    """Pinned host buffer sets handed out inside :class:`DeviceResult` objects.

    A set is reused only once the DeviceResult that last carried it has been dropped by its
    consumer (tracked with a weak reference) — a consumer holding many results in flight never
    sees its data overwritten: the ring grows instead (up to ``max_sets``, then raises).  Before
    a set is rewritten the current stream waits for the copy that last wrote it (its event), so
    an abandoned result's late copy cannot land on top of the new one.
    """

    def __init__(self, factory, initial: int = 4, max_sets: int = 256):
        self._factory = factory
        self._sets = [factory() for _ in range(max(1, initial))]
        self._holders = [None] * len(self._sets)       # weakref to the DeviceResult, or None
        self._events = [None] * len(self._sets)
        self._cursor = 0
        self.max_sets = max_sets

    def __len__(self):
        return len(self._sets)

    def acquire(self):
        """(index, buffers) of a set no live DeviceResult refers to."""
        n = len(self._sets)
        for i in range(n):
            idx = (self._cursor + i) % n
            ref = self._holders[idx]
            if ref is None or ref() is None:
                break
        else:
            if n >= self.max_sets:
                raise RuntimeError(f"HostRing: {n} results still held by consumers (max {self.max_sets}); "
                                   "consume (drop) DeviceResults before requesting more")
            self._sets.append(self._factory())
            self._holders.append(None)
            self._events.append(None)
            idx = n
        self._cursor = (idx + 1) % len(self._sets)
        ev = self._events[idx]
        if ev is not None:
            torch.cuda.current_stream().wait_event(ev)
        return idx, self._sets[idx]

    def bind(self, idx: int, result: "DeviceResult") -> "DeviceResult":
        self._holders[idx] = weakref.ref(result)
        self._events[idx] = result.event
        return result


_STREAMS: dict = {}


def named_stream(name: str, device) -> "torch.cuda.Stream":
    """One HIP stream per (device, name), shared by the elements that name it."""
    key = (str(device), name)
    st = _STREAMS.get(key)
    if st is None:
        st = _STREAMS[key] = torch.cuda.Stream(device=device)
    return st


class CapturedCall:
    """hipGraph capture of ``fn(*static_inputs)`` for one input signature.  ``static=True``
    captures against the given input tensors themselves (stable FramePool slot addresses):
    replays then read the producer's buffer directly, no input copy."""

    def __init__(self, fn, example_inputs, warmup: int = 1, static: bool = False):
        self.static_inputs = list(example_inputs) if static else [t.clone() for t in example_inputs]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.static_outputs = fn(*self.static_inputs)
        outs = self.static_outputs if isinstance(self.static_outputs, (tuple, list)) else (self.static_outputs,)
        self._out_ptrs = [t.data_ptr() for t in outs if isinstance(t, torch.Tensor)]
        _STABLE_PTRS.update(self._out_ptrs)

    def drop(self):
        """Forget this graph (LRU eviction): its static outputs stop counting as stable."""
        _STABLE_PTRS.difference_update(self._out_ptrs)
        self.graph = None

    def __call__(self, *inputs):
        for dst, src in zip(self.static_inputs, inputs):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_outputs

    def graph_replay(self):
        self.graph.replay()
        return self.static_outputs


class GpuPipelineElement(PipelineElement):
    """Base class: resolves the device, offers ``run_maybe_captured(key, fn, *inputs)``."""

    def __init__(self, context):
        context.get_implementation("PipelineElement").__init__(self, context)
        deploy = getattr(self.definition, "deploy", None)
        device_spec = getattr(deploy, "device", None)
        device_param, found = self.get_parameter("device")
        if found:
            device_spec = device_param
        if str(device_spec) != "cpu":       # CPU only when asked for explicitly (gloo tests)
            require_gpu()
        self.device = parse_device(device_spec)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        self.gpu_config = get_gpu_configuration()
        graph, _ = self.get_parameter("graph", default=self.gpu_config.graph)
        self.use_graph = str(graph).lower() in ("true", "1", "yes")
        # optional dedicated HIP stream (parameter "hip_stream": name): independent graph branches
        # on different streams run concurrently on the GPU; joins use events
        stream_name, found = self.get_parameter("hip_stream")
        self.hip_stream = named_stream(str(stream_name), self.device) if found and stream_name \
            and self.device.type == "cuda" else None
        self.hip_stream_name = str(stream_name) if self.hip_stream is not None else "default"
        self._captured: dict = {}
        self.share["device"] = str(self.device)
        self._telemetry = {"frames": 0, "t0": time.perf_counter(), "t_last": 0.0, "n_last": 0}

    def load_model_weights(self, model):
        """Element parameter ``weights``: a safetensors file written by ``model.save()`` (packed
        weights + fp8 scale tables); without it the model keeps its seeded random init."""
        path, found = self.get_parameter("weights")
        if found and path:
            model.load(str(path))
            self.share["weights"] = str(path)
        return model

    # set True by elements whose mutable device state is keyed by the frame lane
    lane_safe = False

    @property
    def lane(self) -> int:
        """Frame lane of the frame being processed (``gpu/lanes.py``; 0 without lanes)."""
        from .lanes import current_lane
        return current_lane()

    # per-address graphs kept per (key, lane) — least recently used evicted beyond this
    max_graphs_per_key = 16
    # addresses remembered (LRU) while waiting to recur
    max_seen_addresses = 64

    def run_maybe_captured(self, key, fn, *inputs):
        """Replay a hipGraph of ``fn`` for this input signature and lane, captured on the input
        buffers themselves (one graph per input address — FramePool slots and element rings
        cycle through a few — no per-frame input copy).  Per-address graphs are kept LRU,
        ``max_graphs_per_key`` per key; once that many exist, a NEW address gets its own graph
        only if it is known stable (a FramePool slot, an upstream graph's static output) or it
        recurs — a stream of transient buffers runs one graph with copied-in static inputs
        instead of paying a capture each."""
        if not self.use_graph:
            return fn(*inputs)
        base = (key, self.lane)
        addrs = tuple(t.data_ptr() for t in inputs)
        graphs = self._captured.get(("graphs",) + base)
        if graphs is None:
            from collections import OrderedDict
            graphs = self._captured[("graphs",) + base] = OrderedDict()
            self._captured[("seen",) + base] = OrderedDict()
        call = graphs.get(addrs)
        if call is not None:
            graphs.move_to_end(addrs)
            return call.graph_replay()
        seen = self._captured[("seen",) + base]
        if (_ADMIT_ALL or len(graphs) < self.max_graphs_per_key or addrs in seen
                or all(a in _STABLE_PTRS for a in addrs)):
            seen.pop(addrs, None)
            call = graphs[addrs] = CapturedCall(fn, inputs, static=True)
            if len(graphs) > self.max_graphs_per_key:
                self._retire_graph(graphs.popitem(last=False)[1])
            return call.graph_replay()
        seen[addrs] = True
        if len(seen) > self.max_seen_addresses:
            seen.popitem(last=False)
        call = self._captured.get(base)
        if call is None:
            call = CapturedCall(fn, inputs)
            self._captured[base] = call
        return call(*inputs)

    def _retire_graph(self, call: "CapturedCall") -> None:
        """An evicted graph is destroyed only once the GPU is past its last replay."""
        ev = torch.cuda.Event()
        ev.record()
        graveyard = self._captured.setdefault(("retired",), [])
        graveyard[:] = [(e, c) for e, c in graveyard if not e.query() or c.drop()]
        graveyard.append((ev, call))

    def hold_for_frame(self, pool: "FramePool", slot: int) -> None:
        """Keep ``slot`` of ``pool`` until the frame being processed completes, then release it
        once the GPU is done with the frame (``FramePool.release_after``)."""
        frame = self.pipeline.current_frame() if self.pipeline is not None else None
        if frame is None:
            pool.release_after(slot)
        else:
            frame.on_complete.append(lambda: pool.release_after(slot))

    def stream_enter(self, frame):
        """Engine hook before process_frame: order this element after the producers of its
        inputs (events recorded by side-stream elements) and switch to its own stream."""
        events = getattr(frame, "_hip_events", None)
        target = self.hip_stream
        if events:
            wait_on = target if target is not None else torch.cuda.current_stream(self.device)
            for io in self.definition.input or []:
                ev = events.get(io["name"])
                if ev is not None:
                    wait_on.wait_event(ev)
        if target is None:
            return None
        target.wait_stream(torch.cuda.current_stream(self.device))   # fork point: prior work
        ctx = torch.cuda.stream(target)
        ctx.__enter__()
        return ctx

    def stream_exit(self, frame, outputs, ctx):
        if ctx is None:
            return
        ev = torch.cuda.Event()
        ev.record(self.hip_stream)
        ctx.__exit__(None, None, None)
        if not hasattr(frame, "_hip_events"):
            frame._hip_events = {}
            frame._hip_pending = []
            device = self.device

            def join():   # end of frame: the default stream sees every side stream's work
                cur = torch.cuda.current_stream(device)
                for e in frame._hip_pending:
                    cur.wait_event(e)
            frame._hip_join = join
        for name in (outputs or {}):
            frame._hip_events[name] = ev
        frame._hip_pending.append(ev)

    def frame_done(self, seconds: float) -> None:
        """Engine hook after each local process_frame: GPU telemetry in the EC share (at most
        once a second, so dashboards see frames/s, host-side ms/frame and HBM use per element)."""
        t = self._telemetry
        t["frames"] += 1
        now = time.perf_counter()
        if now - t["t_last"] < 1.0:
            return
        from ..parallel import dist as D
        comm = D.comm_bytes_total()
        if t["t_last"]:
            dt = now - t["t_last"]
            self.share["gpu_fps"] = round((t["frames"] - t["n_last"]) / dt, 1)
            if comm:
                self.share["rccl_mb"] = round(comm / 2**20, 1)
                self.share["rccl_gbps"] = round((comm - t.get("comm_last", 0)) / dt / 1e9, 3)
        t["t_last"], t["n_last"], t["comm_last"] = now, t["frames"], comm
        self.share["gpu_frames"] = t["frames"]
        self.share["gpu_host_ms"] = round(seconds * 1e3, 3)
        if self.device.type == "cuda":
            self.share["hbm_allocated_mb"] = round(torch.cuda.memory_allocated(self.device) / 2**20, 1)
            self.share["hbm_reserved_mb"] = round(torch.cuda.memory_reserved(self.device) / 2**20, 1)
        pool = getattr(self, "frame_pool", None)
        if pool is not None:
            self.share["frame_pool_free"] = pool.free_count()

    def gpu_timer_start(self):
        """HIP event on the element's stream (the engine calls this after ``stream_enter``)."""
        if self.device.type != "cuda":
            return None
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        return start

    def gpu_timer_stop(self, start):
        end = torch.cuda.Event(enable_timing=True)
        end.record()
        start._aiko_end = end
        return end

    def start_stream(self, stream, stream_id):
        return StreamEvent.OKAY, None
