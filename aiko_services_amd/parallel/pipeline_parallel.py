"""Pipeline parallelism: one aiko Pipeline stage per GPU, stage hand-off by RCCL P2P over xGMI.

BASELINE config 3 ("4-stage video pipeline decode -> resize -> ResNet-50 -> postprocess
pipeline-parallel across 4 MI355X").  Every rank (one process per GPU, ``torchrun``) builds
only the elements of its stage — ``deploy.local.stage`` in the PipelineDefinition, or an even
split of the element chain — as an ordinary local aiko Pipeline, then runs a frame loop:

    rank 0:       frame -> local stage -> send(boundary tensors) -> rank 1
    rank r:       recv -> local stage -> send -> rank r+1
    last rank:    recv -> local stage -> output (DeviceResult / response queue)

Hand-off protocol (``StageLink``): the first frame of a stream carries a signature header
(names, dtypes, shapes) so the receiver allocates its HBM receive slots once; afterwards each
frame is a small int64 header (frame id, stream state) plus the tensors, posted as one grouped
``batch_isend_irecv``.  Send and receive slots are rings of ``depth`` buffers: the sender copies
its boundary tensors into a slot (device-to-device, never via the host) and returns while RCCL
moves them, so stage r computes frame k+1 while frame k is on the xGMI link; a slot is reused
only after its transfer completed.  MQTT never carries tensor payloads.  Stream state (DROP /
STOP / ERROR) travels in the header; intermediate stages forward it without a host sync and
the last stage discards dropped frames.
"""
from __future__ import annotations

import copy
from collections import OrderedDict
import queue
import time

import torch

from ..pipeline.definition import PipelineDefinition
from ..utils.graph import Graph, Node
from . import dist as D

__all__ = ["StageLink", "element_chain", "split_stages", "stage_definition", "boundary_names",
           "PipelineParallelRunner", "HEADER"]

_DTYPES = [torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.float16,
           torch.float32, torch.float64, torch.bfloat16, torch.bool]
HEADER = 4          # int64 [frame_id, stream_state, t_submit_ns, reserved]
_MAX_DIMS = 6


def element_chain(definition: PipelineDefinition):
    """Element names in the engine's execution order for the (single) graph path.  Elements
    exchange data through the frame's swag, so any execution order can be cut into stages."""
    heads, successors = Graph.traverse(definition.graph)
    if len(heads) != 1:
        raise ValueError("pipeline parallelism needs exactly one graph path")
    graph = Graph(heads)
    for name, succ in successors.items():
        graph.add(Node(name, None, OrderedDict(succ)))
    return [node.name for node in graph.get_path()]


def split_stages(definition: PipelineDefinition, num_stages: int):
    """Element names per stage: ``deploy.local.stage`` when every element has one, else an
    even split of the chain (earlier stages take the remainder)."""
    order = element_chain(definition)
    by_name = {e.name: e for e in definition.elements}
    explicit = [getattr(by_name[n].deploy, "stage", None) for n in order]
    if all(s is not None for s in explicit):
        stages = [[] for _ in range(num_stages)]
        last = 0
        for n, s in zip(order, explicit):
            s = int(s)
            if not 0 <= s < num_stages:
                raise ValueError(f"element {n}: stage {s} outside 0..{num_stages - 1}")
            if s < last:
                raise ValueError(f"element {n}: stage {s} precedes stage {last} of its predecessor")
            last = s
            stages[s].append(n)
    else:
        n, k = len(order), num_stages
        sizes = [n // k + (1 if i < n % k else 0) for i in range(k)]
        stages, at = [], 0
        for size in sizes:
            stages.append(order[at:at + size])
            at += size
    if any(not s for s in stages):
        raise ValueError(f"cannot place {len(order)} elements on {num_stages} stages: {stages}")
    return stages


def stage_definition(definition: PipelineDefinition, names) -> PipelineDefinition:
    """A standalone PipelineDefinition holding only ``names`` (chained in order)."""
    elements = [copy.deepcopy(e) for e in definition.elements if e.name in names]
    return PipelineDefinition(version=definition.version, name=f"{definition.name}_{names[0]}",
                              runtime=definition.runtime, graph=[f"({' '.join(names)})"],
                              parameters=dict(definition.parameters), elements=elements)


def boundary_names(definition: PipelineDefinition, stages, rank: int):
    """Swag names stage ``rank`` must forward: produced at stages <= rank (or received) and
    consumed by an input of a later stage."""
    by_name = {e.name: e for e in definition.elements}
    produced, consumed = set(), set()
    for r, names in enumerate(stages):
        for n in names:
            if r <= rank:
                produced.update(o["name"] for o in by_name[n].output)
            else:
                consumed.update(i["name"] for i in by_name[n].input)
    return [n for n in sorted(produced & consumed)]


class StageLink:
    """One direction of a stage boundary: a ring of ``depth`` HBM slots (header + tensors)."""

    def __init__(self, peer: int, device, depth: int = 2):
        if depth < 2:
            # the receiver posts frame k+1's receive before frame k's compute is queued; with a
            # single slot that receive would overwrite the inputs frame k is still reading
            raise ValueError(f"StageLink depth must be >= 2 (got {depth}): one slot in use by the "
                             "stage, one receiving the next frame")
        self.peer = peer
        self.device = torch.device(device)
        self.depth = depth
        self.signature = None           # [(name, dtype, shape)]
        self.slots = []                 # [(header, {name: tensor})]
        self.pending = [None] * self.depth
        self.cursor = 0
        self.bytes_per_frame = 0

    # ---- signature exchange (first frame of the stream only) -----------------------------------
    def _alloc(self):
        self.slots = []
        for _ in range(self.depth):
            hdr = torch.zeros(HEADER, dtype=torch.int64, device=self.device)
            bufs = {n: torch.empty(shape, dtype=dt, device=self.device) for n, dt, shape in self.signature}
            self.slots.append((hdr, bufs))
        self.bytes_per_frame = sum(t.numel() * t.element_size() for t in self.slots[0][1].values())

    def send_signature(self, tensors: dict):
        self.signature = [(n, t.dtype, tuple(t.shape)) for n, t in tensors.items()]
        enc = [len(self.signature)]
        for _n, dt, shape in self.signature:
            if len(shape) > _MAX_DIMS:
                raise ValueError(f"stage boundary tensors support <= {_MAX_DIMS} dims")
            enc += [_DTYPES.index(dt), len(shape)] + list(shape) + [0] * (_MAX_DIMS - len(shape))
        blob = "\x00".join(n for n, _, _ in self.signature).encode()
        enc.append(len(blob))
        meta = torch.tensor(enc, dtype=torch.int64, device=self.device)
        D.send(torch.tensor([meta.numel()], dtype=torch.int64, device=self.device), self.peer)
        D.send(meta, self.peer)
        if blob:
            D.send(torch.tensor(list(blob), dtype=torch.uint8, device=self.device), self.peer)
        self._alloc()

    def recv_signature(self):
        size = torch.zeros(1, dtype=torch.int64, device=self.device)
        D.recv(size, self.peer)
        meta = torch.zeros(int(size.item()), dtype=torch.int64, device=self.device)
        D.recv(meta, self.peer)
        m = meta.tolist()
        count, off, sig = m[0], 1, []
        for _ in range(count):
            dt, nd = _DTYPES[m[off]], m[off + 1]
            sig.append((dt, tuple(m[off + 2:off + 2 + nd])))
            off += 2 + _MAX_DIMS
        nblob, names = m[off], []
        if nblob:
            blob = torch.zeros(nblob, dtype=torch.uint8, device=self.device)
            D.recv(blob, self.peer)
            names = bytes(blob.tolist()).decode().split("\x00")
        self.signature = [(n, dt, shape) for n, (dt, shape) in zip(names, sig)]
        self._alloc()

    # ---- frames --------------------------------------------------------------------------------
    def _retire(self, slot):
        for w in self.pending[slot] or []:
            w.wait()            # RCCL: current stream waits on the P2P stream (no host block)
        self.pending[slot] = None

    def send(self, header, tensors: dict):
        """``header``: device int64[HEADER] tensor or a list of ints.  Copies into the next slot
        (so the producer may overwrite its buffers) and posts the grouped send."""
        if self.signature is None:
            self.send_signature(tensors)
        slot = self.cursor
        self.cursor = (slot + 1) % self.depth
        self._retire(slot)
        hdr, bufs = self.slots[slot]
        if isinstance(header, torch.Tensor):
            hdr.copy_(header, non_blocking=True)
        else:
            hdr.copy_(torch.tensor(list(header) + [0] * (HEADER - len(header)), dtype=torch.int64))
        for n, dt, shape in self.signature:
            t = tensors.get(n)
            if t is None:           # dropped frame without outputs: header state says so
                continue
            if t.dtype != dt or tuple(t.shape) != shape:
                raise ValueError(f"stage boundary '{n}' changed from {dt}{shape} to {t.dtype}{tuple(t.shape)}"
                                 " within a stream")
            bufs[n].copy_(t, non_blocking=True)
        ops = [("send", hdr, self.peer)] + [("send", bufs[n], self.peer) for n, _, _ in self.signature]
        self.pending[slot] = D.batch_p2p(ops)

    def post_recv(self):
        """Post the receive of the next frame into the next slot; returns the slot index."""
        if self.signature is None:
            self.recv_signature()
        slot = self.cursor
        self.cursor = (slot + 1) % self.depth
        self._retire(slot)
        hdr, bufs = self.slots[slot]
        ops = [("recv", hdr, self.peer)] + [("recv", bufs[n], self.peer) for n, _, _ in self.signature]
        self.pending[slot] = D.batch_p2p(ops)
        return slot

    def wait(self, slot):
        self._retire(slot)
        return self.slots[slot]

    def drain(self):
        for slot in range(self.depth):
            self._retire(slot)


class StageFailure(RuntimeError):
    """A neighbouring stage rank is gone (transport error on its link)."""

    def __init__(self, peer: int, cause: BaseException):
        super().__init__(f"pipeline-parallel stage rank {peer} failed: {cause}")
        self.peer = peer


class PipelineParallelRunner:
    """This rank's stage of a pipeline-parallel PipelineDefinition.

    ``step(frame_data)`` advances one frame: stage 0 takes ``frame_data`` (usually empty: its
    first element generates frames), later stages receive from their predecessor.  The last
    stage returns ``(stream_info, outputs)``; earlier stages return None.  Receives are posted
    one frame ahead so the xGMI transfer of frame k+1 overlaps this stage's compute of frame k.
    """

    def __init__(self, definition: PipelineDefinition, device=None, depth: int | None = None,
                 stream_id: str = "pp"):
        from ..pipeline.engine import PipelineImpl
        self.rank, self.world = D.rank(), D.world_size()
        if depth is None:
            from ..utils.configuration import get_gpu_configuration
            depth = get_gpu_configuration().pp_depth
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        self.device = torch.device(device)
        self.stages = split_stages(definition, self.world)
        self.names = self.stages[self.rank]
        self.definition = stage_definition(definition, self.names)
        self.stream_id = stream_id
        self.responses: queue.Queue = queue.Queue()
        self.pipeline = PipelineImpl.create_pipeline(
            "<pipeline_parallel>", self.definition, f"{definition.name}_stage{self.rank}", None,
            stream_id, [], 0, None, 3600, queue_response=self.responses)
        self.pipeline.response_swag = True      # responses carry the whole swag, not just the tail
        self.prev = StageLink(self.rank - 1, self.device, depth) if self.rank > 0 else None
        self.next = StageLink(self.rank + 1, self.device, depth) if self.rank < self.world - 1 else None
        self.boundary = boundary_names(definition, self.stages, self.rank)
        self.frame_id = 0
        self._posted = None                  # slot of the receive posted ahead
        self._host_hdr = None
        self._host_slot = 0
        self._state_hdr = torch.zeros(HEADER, dtype=torch.int64, device=self.device)
        self.healthy = True
        self.failed_peer = None

    @property
    def is_first(self):
        return self.prev is None

    @property
    def is_last(self):
        return self.next is None

    def _host_header(self, hdr):
        """Asynchronous copy of a received header to a pinned host ring (read after the frame's
        results have been waited for — never forces a sync here)."""
        if self.device.type != "cuda":
            return hdr.clone()
        if self._host_hdr is None:
            self._host_hdr = [torch.zeros(HEADER, dtype=torch.int64, pin_memory=True) for _ in range(16)]
        h = self._host_hdr[self._host_slot]
        self._host_slot = (self._host_slot + 1) % len(self._host_hdr)
        h.copy_(hdr, non_blocking=True)
        return h

    def _link_failed(self, peer: int, exc: BaseException):
        """Health: a transport error on a stage link marks the peer absent — the
        stage pipeline's lifecycle drops to "waiting" and its share names the failed rank — and
        surfaces as ``StageFailure`` to the caller (which ends or re-forms the stream).  On RCCL
        a dead peer shows up as a communicator error / watchdog timeout on the next wait; on
        gloo as a closed connection."""
        self.healthy = False
        self.failed_peer = peer
        share = getattr(self.pipeline, "ec_producer", None)
        if share is not None:
            share.update("lifecycle", "waiting")
            share.update("stage_failed", peer)
        raise StageFailure(peer, exc) from exc

    def _recv_next(self):
        try:
            slot = self._posted if self._posted is not None else self.prev.post_recv()
            in_hdr, bufs = self.prev.wait(slot)
            self._posted = self.prev.post_recv()      # next frame's transfer overlaps our compute
        except RuntimeError as exc:
            self._link_failed(self.rank - 1, exc)
        return in_hdr, bufs

    def step(self, frame_data=None):
        if not self.healthy:
            raise StageFailure(self.failed_peer, RuntimeError("stage link already failed"))
        frame_data = dict(frame_data or {})
        in_hdr = upstream = None
        if self.prev is not None:
            in_hdr, bufs = self._recv_next()
            frame_data.update(bufs)
            if self.is_last:
                host = self._host_header(in_hdr)
                frame_data["t_submit"] = host[2:3]
                upstream = host
        self.pipeline.process_frame({"stream_id": self.stream_id, "frame_id": self.frame_id}, frame_data)
        info, out = self.responses.get_nowait()
        fid = self.frame_id
        self.frame_id += 1
        if self.next is not None:
            tensors = {n: out[n] for n in self.boundary if isinstance(out.get(n), torch.Tensor)}
            if in_hdr is None:
                t = out.get("t_submit", frame_data.get("t_submit", time.perf_counter()))
                header = [fid, int(info["state"]), int(float(t) * 1e9), 0]
            else:
                header = self._state_hdr
                header.copy_(in_hdr, non_blocking=True)
                if int(info["state"]) != 0:
                    header[1] = int(info["state"])
            try:
                self.next.send(header, tensors)
            except RuntimeError as exc:
                self._link_failed(self.rank + 1, exc)
            return None
        if upstream is not None:
            # pinned int64 [frame_id, state, t_submit_ns, 0] of the frame as sent by stage 0 and
            # folded by every stage; read it after the frame's results are complete
            info = dict(info, header=upstream)
        return info, out

    @staticmethod
    def upstream_state(info) -> int:
        """Stream state a frame had on the earlier stages (0 = RUN, 1 = DROP_FRAME, ...)."""
        h = info.get("header")
        return 0 if h is None else int(h[1])

    def finish(self):
        """End of stream, called on every rank after its last ``step``: the look-ahead receive
        each later stage posted is matched by a terminator frame (state -1) that flows down the
        chain, then all outstanding transfers complete."""
        if self.prev is not None and self._posted is not None:
            self.prev.wait(self._posted)
            self._posted = None
        if self.next is not None and self.next.signature is not None:
            _, bufs = self.next.slots[self.next.cursor]
            self.next.send([self.frame_id, -1, 0, 0], dict(bufs))
            self.next.drain()
        if self.prev is not None:
            self.prev.drain()
