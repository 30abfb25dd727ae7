"""Placement of one PipelineDefinition over the GPUs of a node: stages, replicas, ranks.

The reference spreads a pipeline over processes by hand: each process runs its own definition
and a parent reaches the next one through a ``remote`` element found by the registrar
(``/root/reference/src/aiko_services/examples/pipeline/multitude/pipeline_small_a.json``,
``run_large.sh``).  Here the same nested-remote topology is GENERATED from one definition
annotated with ``"parallel": {"mode": "pp", "gpus": N}`` and/or ``deploy.local.stage``:

* the element chain is cut into stages (explicit ``stage`` indices, or the planner below);
* stage ``s`` runs as Pipeline ``{name}_s{s}`` (stage 0 keeps ``name``: it is the pipeline
  ``aiko_pipeline create`` started) whose graph ends in a remote element standing for stage
  ``s + 1`` — exactly the reference's chained remote pipelines, the response of the last stage
  flowing back up the chain as ``process_frame_response``;
* a stage may be REPLICATED on several GPUs (PP x DP): every replica registers under the same
  service name with tags ``rank=r`` / ``weight=w`` and the upstream stage spreads frames over
  them (``RemoteReplicas``, weighted round-robin).  ``local_share`` > 0 also runs a copy of
  the LAST stage inside rank 0 (its GPU would otherwise only feed the others);
* every process is one rank of one RCCL group; ``links`` lists the (src, dst) directions the
  hop data plane needs (``parallel/hop.py``).

``plan_stages`` is the balancer: from measured per-element GPU times (``frame.metrics
["gpu_events"]`` of a 1-GPU run, or ``bench.py --profile-elements``) it picks the cut points,
replica counts and rank-0 share that minimise the slowest rank's time per frame.
"""
from __future__ import annotations

import copy
import itertools
import json
import uuid
from dataclasses import asdict, dataclass, field

from ..pipeline.definition import parse_pipeline_definition_dict

__all__ = ["Plan", "RankSpec", "plan_stages", "make_plan", "ingest_ms_of", "size_hop_batch", "hop_pairs_per_s", "HOP_CEILING_FPS", "element_chain", "element_order", "predicted_times",
           "boundary_ms_from_bytes",
           "stage_remote_name"]


@dataclass
class RankSpec:
    rank: int
    stage: int
    name: str                  # Pipeline (service) name this rank registers
    definition: dict           # PipelineDefinition (JSON dict) this rank runs
    device: int                # local GPU index
    weight: float = 1.0        # share of its stage's frames (replicas)
    tags: list = field(default_factory=list)


@dataclass
class Plan:
    group: str
    world: int
    mode: str
    stages: list               # [[element names]]
    replicas: list             # ranks per stage
    local_share: float         # fraction of the last stage's frames run inside rank 0
    ranks: list                # [RankSpec]
    links: list                # [[src, dst]] hop directions (one RCCL communicator each)
    predicted_ms: dict = field(default_factory=dict)
    stream: dict = field(default_factory=dict)   # dp: every rank creates this stream
    stage_defs: list = field(default_factory=list)   # PipelineDefinition (JSON) of every stage

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, text: str) -> "Plan":
        d = json.loads(text)
        d["ranks"] = [RankSpec(**r) for r in d["ranks"]]
        return cls(**d)


def element_chain(definition) -> list:
    """Element names of a parsed PipelineDefinition in the engine's execution order for its
    (single) graph path.  Elements exchange data through the frame's swag, so any execution
    order can be cut into stages."""
    from collections import OrderedDict
    from ..utils.graph import Graph, Node
    heads, successors = Graph.traverse(definition.graph)
    if len(heads) != 1:
        raise ValueError("pipeline parallelism needs exactly one graph path")
    graph = Graph(heads)
    for name, succ in successors.items():
        graph.add(Node(name, None, OrderedDict(succ)))
    return [node.name for node in graph.get_path()]


def element_order(definition: dict):
    return element_chain(parse_pipeline_definition_dict(definition))


def stage_remote_name(base: str, stage: int) -> str:
    return base if stage == 0 else f"{base}_s{stage}"


# ---- balancer ---------------------------------------------------------------------------------

def predicted_times(stages_ms, replicas, local_share=0.0):
    """Per-rank ms per frame: stage s's time split over its replicas; rank 0 also runs
    ``local_share`` of the last stage."""
    per_rank = []
    last = len(stages_ms) - 1
    for s, (t, r) in enumerate(zip(stages_ms, replicas)):
        if s == last and last > 0:
            remote = (1.0 - local_share) * t
            per_rank += [remote / r] * r
        else:
            per_rank += [t / r] * r
    if last > 0:
        per_rank[0] += local_share * stages_ms[last]
    return per_rank


def plan_stages(order, times_ms: dict, gpus: int, replicate: bool = True, local: bool = True,
                boundary_ms: dict | None = None):
    """Best (stages, replicas, local_share, per-rank ms) for ``gpus`` ranks.

    ``order``: element names in execution order; ``times_ms``: measured GPU ms per frame of
    each element on one GPU; ``boundary_ms[name]`` (optional): cost of shipping the swag after
    element ``name`` to the next stage, added to the receiving stage.  Stage 0 has one rank
    (the source); later stages may be replicated.  Exhaustive over cut points and replica
    splits (chains are short: 2^(n-1) cuts x compositions of ``gpus``)."""
    n = len(order)
    boundary_ms = boundary_ms or {}
    best = None
    for cuts in itertools.product([0, 1], repeat=n - 1):
        stages, cur = [], [order[0]]
        for name, cut in zip(order[1:], cuts):
            if cut:
                stages.append(cur)
                cur = []
            cur.append(name)
        stages.append(cur)
        S = len(stages)
        if S > gpus:
            continue
        t = []
        for s, names in enumerate(stages):
            ms = sum(float(times_ms.get(e, 0.0)) for e in names)
            if s > 0:
                ms += float(boundary_ms.get(stages[s - 1][-1], 0.0))
            t.append(ms)
        splits = [[1] * S]
        if replicate and S > 1:
            splits = [list(c) for c in _compositions(gpus, S) if c[0] == 1]
        for reps in splits:
            if sum(reps) > gpus:
                continue
            shares = [0.0]
            if local and S == 2 and t[1] > 0:
                # rank 0 hosts a copy of stage 1 taking share s of its frames: balanced when
                # t0 + s * t1 == (1 - s) * t1 / r1
                r1 = reps[1]
                shares.append(min(0.95, max(0.0, (t[1] - r1 * t[0]) / (t[1] * (1 + r1)))))
            for share in shares:
                per_rank = predicted_times(t, reps, share)
                key = (round(max(per_rank), 6), len(per_rank), -share)
                if best is None or key < best[0]:
                    best = (key, stages, reps, share, per_rank)
    _, stages, reps, share, per_rank = best
    return stages, reps, share, per_rank


def plan_ingest(order, times_ms: dict, gpus: int, ingest_ms: float, boundary_ms: dict | None = None):
    """Where frames enter HBM when they come from the host (decode / camera / files): the
    PCIe term of the balancer.  ``ingest_ms`` = upload time of one frame batch over one
    rank's PCIe link.

    * ``rank0``: the source stage on rank 0 decodes AND uploads every batch of the node (its
      time grows by ``ingest_ms`` per batch) and the stage cut ships frames over xGMI — the
      best :func:`plan_stages` plan with that cost;
    * ``per_rank``: every rank decodes and uploads its own batches over its own PCIe link
      (data parallel: the whole chain per rank, nothing crosses xGMI): per-rank time per node
      batch = (chain + ingest) / gpus.

    Returns ``(choice, per-rank ms, plan_stages result or None)``: the choice with the lower
    busiest-rank time (ms per frame batch of the node)."""
    times0 = dict(times_ms)
    times0[order[0]] = float(times0.get(order[0], 0.0)) + float(ingest_ms)
    pp = plan_stages(order, times0, gpus, boundary_ms=boundary_ms)
    rank0_ms = max(pp[3])
    chain = sum(float(times_ms.get(e, 0.0)) for e in order) + float(ingest_ms)
    per_rank_ms = chain / max(1, gpus)
    if per_rank_ms < rank0_ms:
        return "per_rank", [per_rank_ms] * gpus, None
    return "rank0", pp[3], pp


# Control-plane ceiling: frames/s that rank 0's event loop sustains through remote hops (one
# process_frame + process_frame_response pair per message, a message carrying ``hop_batch``
# frames), flat out, 8-rank shape (7 replicas), measured on the MI355X box's CPUs with
# ``tools/hop_bench.py`` — profiles/hop_bench_r5_flat_b{1,2,4,8}.json.
HOP_CEILING_FPS = {1: 3502.0, 2: 7013.0, 4: 9836.0, 8: 10711.0}
HOP_HEADROOM = 0.6        # plan for at most this fraction of the ceiling


def hop_pairs_per_s(batches_per_s: float, remote_fraction: float) -> float:
    """Remote-hop pairs (frame batches sent to another rank and answered) per second through
    rank 0: the node's frame-batch rate times the share of batches that leave rank 0."""
    return max(0.0, float(batches_per_s)) * min(1.0, max(0.0, float(remote_fraction)))


def size_hop_batch(pairs_per_s: float, ceiling: dict | None = None, headroom: float = HOP_HEADROOM) -> int:
    """Smallest ``hop_batch`` (frames per hop message) whose measured control-plane ceiling
    leaves ``1 / headroom`` room over the rate the plan needs: ``pairs_per_s <= headroom x
    ceiling[k]``.  Larger groups cost latency (frames wait for a group), so the smallest that
    fits wins; if none fits, the largest measured one."""
    ceiling = {int(k): float(v) for k, v in (ceiling or HOP_CEILING_FPS).items()}
    for k in sorted(ceiling):
        if pairs_per_s <= headroom * ceiling[k]:
            return k
    return max(ceiling)


def ingest_ms_of(par: dict) -> float:
    """PCIe upload time of one frame batch (ms) from a ``parallel`` block: ``ingest_ms``, or
    ``frame_bytes`` (bytes per batch uploaded) over ``pcie_gbps`` (GB/s of one rank's link);
    0 when neither is given (frames are born in HBM: nothing to price)."""
    if par.get("ingest_ms") is not None:
        return float(par["ingest_ms"])
    if par.get("frame_bytes") and par.get("pcie_gbps"):
        return float(par["frame_bytes"]) / (float(par["pcie_gbps"]) * 1e9) * 1e3
    return 0.0


def _compositions(total, parts):
    """Positive integer tuples of length ``parts`` summing to at most ``total``."""
    for k in range(parts, total + 1):
        for cut in itertools.combinations(range(1, k), parts - 1):
            edges = (0,) + cut + (k,)
            yield tuple(edges[i + 1] - edges[i] for i in range(parts))


# ---- plan construction -----------------------------------------------------------------------

def _strip_stage(e: dict) -> dict:
    e = copy.deepcopy(e)
    local = e.get("deploy", {}).get("local")
    if isinstance(local, dict):
        local.pop("stage", None)
    return e


def _boundary(defn: dict, stages, s):
    by = {e["name"]: e for e in defn["elements"]}
    produced, consumed = set(), set()
    for r, names in enumerate(stages):
        for n in names:
            if r <= s:
                produced.update(o["name"] for o in by[n]["output"])
            else:
                consumed.update(i["name"] for i in by[n]["input"])
    return sorted(produced & consumed)


def _dp_plan(definition: dict, gpus: int, group: str | None) -> Plan:
    """``mode: dp`` — SPMD data parallelism: every rank runs the WHOLE definition on its GPU
    (registered as ``{name}_r{rank}``), every rank creates the same stream, and the elements'
    collectives (FrameFanout scatter / broadcast, DetectionsGather / ClassifierTopK
    all-gather) pair up frame by frame over RCCL — BASELINE config 4's topology
    (``examples/yolo/yolo_dp8.json``)."""
    base = definition["name"]
    group = group or f"{base}-{uuid.uuid4().hex[:8]}"
    d = {k: copy.deepcopy(v) for k, v in definition.items() if k != "parallel"}
    d["elements"] = [_strip_stage(e) for e in definition["elements"]]
    ranks = []
    for r in range(gpus):
        dr = copy.deepcopy(d)
        dr["name"] = base if r == 0 else f"{base}_r{r}"
        ranks.append(RankSpec(rank=r, stage=0, name=dr["name"], definition=dr, device=r,
                              tags=[f"rank={r}", f"group={group}", "mode=dp"]))
    return Plan(group=group, world=gpus, mode="dp", stages=[element_order(definition)], replicas=[gpus],
                local_share=0.0, ranks=ranks, links=[])


def _dp_replicated_plan(definition: dict, gpus: int, group: str | None) -> Plan:
    """``mode: dp`` + ``replicated: true`` — data parallelism on the replicated-stage
    machinery instead of SPMD collectives: stage 0 = the ingest prefix (through the fan-out
    element, or the source alone) on rank 0; stage 1 = the rest, one replica per other GPU
    plus rank 0's local share (``local_share`` = rank 0's fraction of the frames, default
    1 / gpus: rank 0 detects as much as each replica).  Frames are dealt to replicas by the hop credits; a dead replica's frames are
    re-dispatched to the survivors (``pipeline/engine.py`` ``_replica_lost``) instead of
    hanging a collective, and a restarted one is re-admitted.  The definition's collective
    elements become pass-throughs (pipeline parameter ``spmd`` false: each frame visits one
    replica).  BASELINE config 4's topology with rank loss survivable; plain ``mode: dp``
    keeps the SPMD fast path."""
    par = definition.get("parallel") or {}
    order = element_order(definition)
    by = {e["name"]: e for e in definition["elements"]}

    def cls(n):
        return by[n]["deploy"].get("local", {}).get("class_name") or n
    cut = next((i for i, n in enumerate(order) if cls(n) == "FrameFanout"), 0) + 1
    cut = min(cut, len(order) - 1)
    d = copy.deepcopy(definition)
    d["parameters"] = dict(d.get("parameters") or {}, spmd=False)
    d["parallel"] = {k: v for k, v in par.items() if k not in ("mode", "replicated")}
    d["parallel"]["mode"] = "pp"
    for e in d["elements"]:
        e.get("deploy", {}).get("local", {}).pop("stage", None)
    share = float(par.get("local_share", 1.0 / max(1, gpus)))
    hop = None
    if par.get("times_ms") and gpus > 1:
        # control-plane headroom: each replica (and rank 0's share) runs stage 1 at its measured
        # time per frame batch, so the node completes gpus / t batches per second and the
        # (1 - share) that leave rank 0 are remote-hop pairs through its event loop
        t1 = sum(float(par["times_ms"].get(n, 0.0)) for n in order[cut:])
        if t1 > 0:
            pairs = hop_pairs_per_s(gpus * 1e3 / t1, 1.0 - share)
            k = int(d["parameters"].get("hop_batch") or 0) or size_hop_batch(pairs, par.get("hop_ceiling"))
            d["parameters"]["hop_batch"] = k
            hop = {"hop_pairs_per_s": round(pairs, 1), "hop_batch": k,
                   "hop_ceiling_fps": (par.get("hop_ceiling") or HOP_CEILING_FPS).get(k)}
    plan = make_plan(d, gpus=gpus, stages=[order[:cut], order[cut:]], replicas=[1, max(0, gpus - 1)],
                     local_share=share if gpus > 1 else 1.0, group=group)
    if hop:
        plan.predicted_ms.update(hop)
    return plan


def boundary_ms_from_bytes(boundary_bytes: dict, link_gbps: float) -> dict:
    """Transfer cost of each element's output over one xGMI link: ``bytes / link rate`` (ms
    per frame batch) — the balancer's ``boundary_ms``."""
    return {k: float(v) / (float(link_gbps) * 1e9) * 1e3 for k, v in boundary_bytes.items()}


def make_plan(definition: dict, gpus: int | None = None, stages=None, replicas=None,
              local_share: float = 0.0, times_ms: dict | None = None, group: str | None = None,
              device_offset: int = 0, boundary_ms: dict | None = None) -> Plan:
    """Plan for ``definition`` (a JSON dict).  Stages come from (in order) ``stages``, the
    elements' ``deploy.local.stage``, the balancer (``times_ms`` and ``boundary_ms``: per
    element, the cost of shipping its output to the next stage), or one element per stage."""
    par = definition.get("parallel") or {}
    # (the planner may set pipeline parameters, e.g. hop_batch: never on the caller's dict)
    definition = dict(definition, parameters=dict(definition.get("parameters") or {}))
    mode = par.get("mode", "pp")
    gpus = int(gpus or par.get("gpus", 1))
    ingest = par.get("ingest")
    if mode == "pp" and ingest in ("auto", "per_rank", "rank0") and gpus > 1:
        # host frames (decode / camera / files): where do they enter HBM?  per_rank = every rank
        # ingests its own batches over its own PCIe link and runs the whole chain (SPMD data
        # parallel, nothing on xGMI); rank0 = rank 0 uploads the node's batches and the stage
        # cut ships them over xGMI (its upload time is priced into its stage)
        ims = ingest_ms_of(par)
        times = {k: float(v) for k, v in (times_ms or par.get("times_ms") or {}).items()}
        bnd = boundary_ms if boundary_ms is not None else \
            ({k: float(v) for k, v in par["boundary_ms"].items()} if par.get("boundary_ms") else None)
        choice, per_rank, _ = (plan_ingest(element_order(definition), times, gpus, ims, boundary_ms=bnd)
                               if ingest == "auto" else (ingest, None, None))
        rest = {k: v for k, v in par.items() if k not in ("ingest",)}
        if choice == "per_rank":
            d = dict(definition, parallel=dict(rest, mode="dp"))
            plan = _dp_plan(d, gpus, group)
        else:
            order0 = element_order(definition)
            if times:
                times[order0[0]] = times.get(order0[0], 0.0) + ims
            d = dict(definition, parallel=dict(rest, times_ms=times) if times else rest)
            plan = make_plan(d, gpus=gpus, stages=stages, replicas=replicas, local_share=local_share,
                             group=group, device_offset=device_offset, boundary_ms=boundary_ms)
        plan.predicted_ms.update(ingest=choice, ingest_ms=round(ims, 4))
        if per_rank:
            plan.predicted_ms["ingest_per_rank_ms"] = [round(x, 4) for x in per_rank]
        return plan
    if mode == "dp" and par.get("replicated"):
        return _dp_replicated_plan(definition, gpus, group)
    if mode == "dp":
        return _dp_plan(definition, gpus, group)
    if replicas is None and par.get("replicas") is not None:
        replicas = [int(r) for r in par["replicas"]]
    if not local_share and par.get("local_share") is not None:
        local_share = float(par["local_share"])
    if times_ms is None and par.get("times_ms"):
        times_ms = {k: float(v) for k, v in par["times_ms"].items()}
    if boundary_ms is None and par.get("boundary_ms"):
        boundary_ms = {k: float(v) for k, v in par["boundary_ms"].items()}
    order = element_order(definition)
    by = {e["name"]: e for e in definition["elements"]}
    predicted = {}
    if stages is None:
        explicit = [by[n]["deploy"].get("local", {}).get("stage") for n in order]
        if all(s is not None for s in explicit):
            count = max(int(s) for s in explicit) + 1
            stages = [[] for _ in range(count)]
            for n, s in zip(order, explicit):
                stages[int(s)].append(n)
            stages = [s for s in stages if s]
        elif times_ms:
            stages, replicas, local_share, per_rank = plan_stages(order, times_ms, gpus,
                                                                  boundary_ms=boundary_ms)
            predicted = {"per_rank_ms": [round(x, 4) for x in per_rank]}
            if len(stages) > 1 and max(per_rank) > 0:
                # every frame batch hops once per stage boundary; rank 0 sends the share of the
                # stage-1 batches it does not run itself
                pairs = hop_pairs_per_s(1e3 / max(per_rank), 1.0 - local_share)
                params = definition.setdefault("parameters", {})
                k = int(params.get("hop_batch") or 0) or size_hop_batch(pairs, par.get("hop_ceiling"))
                params["hop_batch"] = k
                predicted.update(hop_pairs_per_s=round(pairs, 1), hop_batch=k)
            if boundary_ms:
                predicted["boundary_ms"] = {s[-1]: round(boundary_ms.get(s[-1], 0.0), 4) for s in stages[:-1]}
        else:
            k = min(gpus, len(order))
            sizes = [len(order) // k + (1 if i < len(order) % k else 0) for i in range(k)]
            stages, at = [], 0
            for size in sizes:
                stages.append(order[at:at + size])
                at += size
    if replicas is None:
        replicas = [1] * len(stages)
    if any(r < 0 for r in replicas) or (replicas[-1] == 0 and not local_share):
        raise ValueError(f"replicas {replicas}: a stage needs a rank or (the last) a local share")
        replicas[-1] += max(0, gpus - sum(replicas)) if par.get("replicate_last", False) else 0
    if len(replicas) != len(stages) or replicas[0] != 1:
        raise ValueError(f"replicas {replicas} must match stages {stages} and start with 1")
    if sum(replicas) > max(gpus, 1):
        raise ValueError(f"plan needs {sum(replicas)} GPUs, only {gpus} given")
    base = definition["name"]
    group = group or f"{base}-{uuid.uuid4().hex[:8]}"
    rank_of_stage, r = [], 0
    for reps in replicas:
        rank_of_stage.append(list(range(r, r + reps)))
        r += reps
    world = r
    last = len(stages) - 1
    ranks = []
    stage_defs = []
    for s, names in enumerate(stages):
        elements = [_strip_stage(by[n]) for n in names]
        graph_names = list(names)
        if s < last:
            remote_name = f"Stage{s + 1}"
            last_el = by[stages[-1][-1]]
            elements.append({
                "name": remote_name,
                "input": [{"name": n, "type": "tensor"} for n in _boundary(definition, stages, s)],
                "output": copy.deepcopy(last_el["output"]),
                "deploy": {"remote": {"module": "aiko_services_amd.pipeline.engine",
                                      "service_filter": {"name": stage_remote_name(base, s + 1)}}},
            })
            graph_names.append(remote_name)
        d = {k: copy.deepcopy(v) for k, v in definition.items() if k not in ("elements", "graph", "parallel")}
        d["name"] = stage_remote_name(base, s)
        # every stage keeps the definition's gpu_lanes: a stage ending in a remote element runs
        # its local prefix on the frame's lane and resumes the response on it (engine Frame.lane);
        # rank 0's local share of the last stage runs in the enclosing frame's lane, so the
        # balancer's element times (measured with lanes) hold on every rank
        d["graph"] = [f"({' '.join(graph_names)})"]
        d["elements"] = elements
        stage_defs.append(d)
        reps = replicas[s]
        for i, rank in enumerate(rank_of_stage[s]):
            w = 1.0
            if s == last and last > 0:
                w = (1.0 - local_share) / reps
            ranks.append(RankSpec(rank=rank, stage=s, name=d["name"], definition=d,
                                  device=device_offset + rank, weight=w,
                                  tags=[f"rank={rank}", f"stage={s}", f"group={group}",
                                        f"weight={w:.6g}"]))
    links = []
    for s in range(last):
        for a in rank_of_stage[s]:
            for b in rank_of_stage[s + 1]:
                links += [[a, b], [b, a]]
    if local_share > 0 and last != 1:
        raise ValueError("local_share needs a two-stage plan (rank 0 hosts a copy of stage 1)")
    return Plan(group=group, world=world, mode=mode, stages=stages, replicas=list(replicas),
                local_share=float(local_share), ranks=ranks, links=links, predicted_ms=predicted,
                stage_defs=stage_defs)
