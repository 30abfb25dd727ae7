"""Multi-GPU actor pipelines: one registered worker Pipeline process per rank of a Plan.

``aiko_pipeline create DEFINITION`` with ``"parallel": {"mode": "pp", "gpus": N}`` (or
``deploy.local.stage`` on the elements) lands here (reference entry point
``/root/reference/src/aiko_services/main/pipeline.py:1444-1528``; multi-process orchestration
in the reference is by hand, ``examples/pipeline/multitude/run_large.sh``):

1. :func:`~aiko_services_amd.parallel.placement.make_plan` cuts the definition into stages,
   replicas and ranks;
2. :func:`spawn_workers` starts ranks 1..N-1 through the :class:`ProcessManager` — BEFORE this
   process touches the GPU — each with ``LOCAL_RANK`` = its GPU, ``RANK`` / ``WORLD_SIZE``
   and the plan file;
3. every rank :func:`join` s: RCCL group bootstrap over the MQTT broker
   (``parallel/rendezvous.py``) and the hop data plane's per-direction communicators
   (``parallel/hop.py``);
4. each worker creates its stage Pipeline, registered with tags ``rank=`` / ``stage=`` /
   ``weight=`` and runs its event loop; rank 0 creates stage 0 (the pipeline the user asked
   for), whose remote element discovers the stage-1 replicas through the registrar.

Frames then flow as in the reference — ``process_frame`` to the remote, ``process_frame_
response`` back — with the tensors on xGMI.  Workers exit when their parent process goes.

Supervision (``AIKO_SUPERVISE=N``: up to N restarts per rank): the ProcessManager's exit
callback restarts a worker that died as a FRESH child process (never an exec of a process that
touched the GPU) with ``AIKO_REJOIN_EPOCH`` / ``AIKO_REJOIN_STORE``.  The restarted rank cannot
join the original default process group, so :func:`rejoin` gives it its identity, announces
``(rejoin rank epoch)`` on ``{namespace}/rendezvous/{group}/rejoin`` and brings its hop links up
as fresh 2-rank groups on the running group's TCPStore; every survivor with a link to it does
its side (:func:`_on_rejoin`), and rank 0's engine re-adds the replica only once those links are
up (reference model: a re-appearing remote is re-bound on the registrar ``add``,
``/root/reference/src/aiko_services/main/pipeline.py:985-1006``; process supervision as in
``/root/reference/src/aiko_services/main/lifecycle.py:144-288``).
"""
from __future__ import annotations

import atexit
import os
import sys
import tempfile
import threading
import time

from .placement import Plan

__all__ = ["spawn_workers", "join", "create_rank_pipeline", "worker_main", "backend_for"]


def backend_for() -> str:
    b = os.environ.get("AIKO_HOP_BACKEND", "auto")
    if b != "auto":
        return b
    import torch
    return "nccl" if torch.cuda.is_available() else "gloo"


def spawn_workers(plan: Plan, plan_path: str | None = None, env: dict | None = None,
                  max_restarts: int | None = None):
    """Start ranks 1..world-1 (``python -m aiko_services_amd.parallel.launch worker``);
    ``max_restarts`` (default ``AIKO_SUPERVISE``, 0) per rank: see the module docstring."""
    from ..control.process_manager import ProcessManager
    if plan_path is None:
        fd, plan_path = tempfile.mkstemp(prefix="aiko_plan_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            f.write(plan.to_json())
    base_env = dict(os.environ if env is None else env)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    base_env["PYTHONPATH"] = root + os.pathsep + base_env.get("PYTHONPATH", "")
    if max_restarts is None:
        max_restarts = int(base_env.get("AIKO_SUPERVISE", "0") or 0)
    # epochs are unique across ranks (one counter): a rank's fresh links are keyed by it
    state = {"stopping": False, "restarts": {}, "epoch": 0}

    def child_env(spec, epoch=0):
        e = dict(base_env, LOCAL_RANK=str(spec.device), RANK=str(spec.rank),
                 WORLD_SIZE=str(plan.world), AIKO_PARENT_PID=str(os.getpid()))
        if epoch:
            from .rendezvous import store_address
            host, port = store_address()
            e.update(AIKO_REJOIN_EPOCH=str(epoch), AIKO_REJOIN_STORE=f"{host}:{port}")
            e.pop("AIKO_FAULTS", None)          # an injected fault is not re-injected
        return e

    def start(spec, epoch=0):
        manager.create(f"rank{spec.rank}", sys.executable,
                       ["-m", "aiko_services_amd.parallel.launch", "worker", plan_path, str(spec.rank)],
                       env=child_env(spec, epoch))

    def on_exit(id, data):
        """ProcessManager monitor thread: a worker exited.  Only a failure is restarted (a
        non-zero or signal exit code); a clean exit is part of a shutdown."""
        if state["stopping"] or not str(id).startswith("rank"):
            return
        if not data.get("return_code"):
            return
        rank = int(str(id)[4:])
        n = state["restarts"].get(rank, 0)
        from .rendezvous import store_address
        if n >= max_restarts or store_address() is None:
            if max_restarts:
                print(f"aiko supervisor: rank {rank} exited ({data.get('return_code')}), not restarted "
                      f"({n} restarts)", file=sys.stderr, flush=True)
            return
        state["restarts"][rank] = n + 1
        state["epoch"] += 1
        print(f"aiko supervisor: rank {rank} exited ({data.get('return_code')}): restarting it, "
              f"epoch {state['epoch']}", file=sys.stderr, flush=True)
        start(plan.ranks[rank], epoch=state["epoch"])

    manager = ProcessManager(process_exit_handler=on_exit)
    manager.supervisor_state = state
    for spec in plan.ranks:
        if spec.rank != 0:
            start(spec)

    def stop():
        state["stopping"] = True
        manager.terminate_all()
    atexit.register(stop)
    atexit.register(lambda: os.path.exists(plan_path) and os.unlink(plan_path))
    return manager, plan_path


def join(plan: Plan, rank: int, timeout_s: float = 120.0):
    """RCCL group over the MQTT broker + the hop data plane (collective: every rank calls)."""
    from ..utils.configuration import get_mqtt_host
    from . import hop
    from .rendezvous import rendezvous_init
    os.environ.setdefault("LOCAL_RANK", str(plan.ranks[rank].device))
    _, host, port = get_mqtt_host()
    backend = backend_for()
    if plan.world > 1:
        rendezvous_init(plan.group, rank, plan.world, host, port, backend=backend, timeout_s=timeout_s)
    depth = int(os.environ.get("AIKO_HOP_DEPTH", "4"))
    plane = hop.init_plane(plan.links, depth=depth)
    _listen_rejoin(plan, plane)

    def report():
        print(f"hop rank {rank} stats: {plane.stats()}", file=sys.stderr, flush=True)
    atexit.register(report)
    return plane


def _rejoin_topic(plan: Plan) -> str:
    from .rendezvous import rendezvous_topic
    return rendezvous_topic(plan.group) + "/rejoin"


def _set_device(plane) -> None:
    """Helper threads that touch the data plane run on the plane's GPU (HIP's current device
    is per thread)."""
    if plane.device.type == "cuda":
        import torch
        torch.cuda.set_device(plane.device)


def _announce(plan: Plan, command: str, rank: int, epoch: int) -> None:
    from ..message.mqtt_client import MQTTClient
    from ..utils.configuration import get_mqtt_host
    from ..utils.sexpr import generate
    _, host, port = get_mqtt_host()
    client = MQTTClient(client_id=f"aiko-{command}-{rank}-{epoch}")
    client.connect(host, port)
    client.publish(_rejoin_topic(plan), generate(command, [rank, epoch]), qos=1, wait=True)
    time.sleep(0.05)
    client.disconnect()


def _listen_rejoin(plan: Plan, plane) -> None:
    """Every rank: on ``(rejoin rank epoch)`` for a peer this rank has links with, bring those
    links up again (off the event loop: it blocks until the peer's side connects), then swap
    them in on the event loop; on ``(rejoined rank epoch)`` — every link of the restarted rank
    is up — let the engine bind it again (:meth:`HopPlane.mark_rejoined`)."""
    from ..runtime import event
    from ..runtime.process import aiko
    from ..utils.sexpr import parse

    def handler(_aiko, _topic, payload):
        try:
            cmd, params = parse(payload)
            peer, epoch = int(params[0]), int(params[1])
        except Exception:                               # noqa: BLE001 — not ours
            return False
        if peer == plane.rank or not plane.links_with(peer):
            return False
        if cmd == "rejoined":
            event.call_soon(plane.mark_rejoined, peer, epoch)
            return False
        if cmd != "rejoin" or plane.epochs.get(peer, 0) >= epoch:
            return False
        # the stage right before the peer's binds it as a remote element: its engine must see
        # the old process's registrar remove (retire links, re-queue held frames) before the
        # fresh links go in.  Any other neighbour (downstream: it only answered the old process)
        # never hears of that death — the announcement itself proves it, so retire them now.
        binds_it = plan.ranks[plane.rank].stage + 1 == plan.ranks[peer].stage
        if not binds_it and peer not in plane.dead:
            event.call_soon(plane.mark_dead, peer)

        def work():
            _set_device(plane)
            deadline = time.time() + 30.0
            while peer not in plane.dead and time.time() < deadline:
                time.sleep(0.05)                        # its death reaches this rank first
            try:
                pending = plane.readmit_connect(peer, epoch)
            except Exception as exc:                    # noqa: BLE001
                print(f"hop rank {plane.rank}: re-admitting rank {peer} failed: {exc}", file=sys.stderr, flush=True)
                return
            event.call_soon(plane.readmit_install, pending)
        threading.Thread(target=work, daemon=True, name=f"hop-readmit-{peer}").start()
        return False
    aiko.process.add_message_handler(handler, _rejoin_topic(plan))


def rejoin(plan: Plan, rank: int, timeout_s: float = 120.0):
    """A restarted rank (``AIKO_REJOIN_EPOCH`` / ``AIKO_REJOIN_STORE``): identity without a
    default process group, a hop plane in rejoin mode, the announcement, then (helper thread)
    its links as fresh 2-rank groups.  The stage pipeline is created meanwhile; the survivors
    only route frames to it once the links are up."""
    from . import dist as D
    from . import hop
    from .rendezvous import connect_store
    os.environ.setdefault("LOCAL_RANK", str(plan.ranks[rank].device))
    epoch = int(os.environ["AIKO_REJOIN_EPOCH"])
    backend = backend_for()
    if backend == "nccl":
        import torch
        torch.cuda.set_device(torch.device("cuda", D.local_rank() % max(1, torch.cuda.device_count())))
    D.set_identity(rank, plan.world, backend)
    store = connect_store(os.environ["AIKO_REJOIN_STORE"], timeout_s)
    depth = int(os.environ.get("AIKO_HOP_DEPTH", "4"))
    plane = hop.init_plane(plan.links, depth=depth, rejoin={"store": store, "epoch": epoch})
    _listen_rejoin(plan, plane)
    _announce(plan, "rejoin", rank, epoch)

    def connect():
        _set_device(plane)
        try:
            peers = plane.connect_rejoin(timeout_s)
            # every link is up: the upstream stage may bind this replica again
            _announce(plan, "rejoined", rank, epoch)
            print(f"hop rank {rank}: re-admitted (epoch {epoch}), links to {peers}", file=sys.stderr, flush=True)
        except Exception as exc:                        # noqa: BLE001
            print(f"hop rank {rank}: rejoin failed: {exc}", file=sys.stderr, flush=True)
    threading.Thread(target=connect, daemon=True, name="hop-rejoin").start()

    def report():
        print(f"hop rank {rank} stats: {plane.stats()}", file=sys.stderr, flush=True)
    atexit.register(report)
    return plane


def create_rank_pipeline(plan: Plan, rank: int, stream_id=None, parameters=None, frame_id=0,
                         frame_data=None, grace_time=60, queue_response=None, name=None,
                         graph_path=None, stream_reset=False, definition_pathname="<parallel>",
                         auto_start=True, extra_tags=()):
    """This rank's stage Pipeline; on rank 0 also binds replicated / local stage members.
    ``auto_start``: a helper thread waits until the stage is ready, joins the start barrier and
    (rank 0) creates the stream — embedders that drive frames themselves pass False."""
    from ..pipeline.definition import parse_pipeline_definition_dict
    from ..pipeline.engine import PipelineImpl
    spec = plan.ranks[rank]
    definition = parse_pipeline_definition_dict(spec.definition)
    if plan.mode == "dp" and rank != 0 and plan.stream:
        # SPMD data parallelism: every rank runs the same stream (its collectives pair up)
        stream_id = plan.stream.get("stream_id")
        parameters = plan.stream.get("parameters") or {}
        grace_time = int(plan.stream.get("grace_time", grace_time))
    pipeline = PipelineImpl.create_pipeline(definition_pathname, definition, name or spec.name, graph_path,
                                            None, [], frame_id, None, grace_time,
                                            queue_response=queue_response, tags=list(spec.tags) + list(extra_tags))
    if plan.mode != "dp" and spec.stage + 1 < len(plan.stages):
        remote = f"Stage{spec.stage + 1}"
        local_def = None
        weight = 0.0
        if spec.stage == 0 and plan.local_share > 0:
            nxt = plan.stage_defs[1] if plan.stage_defs else next(r for r in plan.ranks if r.stage == 1).definition
            local_def = parse_pipeline_definition_dict(nxt)
            weight = plan.local_share
        expected = plan.replicas[spec.stage + 1] + (1 if local_def is not None else 0)
        pipeline.set_remote_replicas(remote, expected, local_def, weight)

    def start():
        from ..runtime.actor import ActorTopic
        if stream_id is not None:
            if stream_reset:
                pipeline._post_message(ActorTopic.IN, "destroy_stream", [stream_id])
            pipeline._post_message(ActorTopic.IN, "create_stream",
                                   [stream_id, None, dict(parameters or {}), grace_time, queue_response, None])
        if frame_data is not None:
            from ..utils.sexpr import parse
            _, arguments = parse(f"(process_frame {frame_data})")
            pipeline.create_frame({"stream_id": stream_id or "*", "frame_id": int(frame_id or 0),
                                   "parameters": {}}, arguments[0])
    if auto_start:
        start_when_ready(pipeline, start if rank == 0 or plan.mode == "dp" else None)
    return pipeline


def start_when_ready(pipeline, then=None, timeout_s: float = 120.0):
    """Helper thread: once this rank's stage is ready (its downstream stages discovered), join
    the group-wide start barrier; rank 0 then creates the stream.  Every stage therefore
    exists, end to end, before the first frame is generated."""
    from . import hop

    def run():
        deadline = time.time() + timeout_s
        while pipeline.share.get("lifecycle") != "ready" and time.time() < deadline:
            time.sleep(0.02)
        plane = hop.plane()
        if plane is not None:
            plane.barrier()
        if then is not None:
            then()
    t = threading.Thread(target=run, daemon=True, name="aiko-parallel-start")
    t.start()
    return t


def _watch_parent():
    """Terminate this worker when the process that spawned it has gone."""
    from ..runtime import event
    from ..runtime.process import aiko
    parent = int(os.environ.get("AIKO_PARENT_PID", "0") or 0)
    if not parent:
        return

    def check():
        try:
            os.kill(parent, 0)
        except OSError:
            aiko.process.terminate(0)
    event.add_timer_handler(check, 0.5)


def _sample_main_thread(path, period=0.005):
    """Statistical profiler of the event-loop thread (cProfile does not see time spent in C
    without a Python frame change): every ``period`` s record the innermost 6 frames."""
    import collections
    import traceback
    main_id = threading.main_thread().ident
    counts = collections.Counter()
    clock = time.pthread_getcpuclockid(main_id)
    start = (time.perf_counter(), time.clock_gettime(clock), os.times())

    def run():
        while True:
            time.sleep(period)
            frame = sys._current_frames().get(main_id)
            if frame is not None:
                stack = traceback.extract_stack(frame)[-6:]
                counts[" <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}"
                                   for f in reversed(stack))] += 1

    def dump():
        with open(path, "w") as f:
            wall = time.perf_counter() - start[0]
            t = os.times()
            f.write(f"wall {wall:.2f}s main-thread cpu {time.clock_gettime(clock) - start[1]:.2f}s "
                    f"process user {t.user - start[2].user:.2f}s sys {t.system - start[2].system:.2f}s\n")
            total = sum(counts.values()) or 1
            for stack, n in counts.most_common(40):
                f.write(f"{100.0 * n / total:5.1f}% {stack}\n")
    threading.Thread(target=run, daemon=True).start()
    atexit.register(dump)


def worker_main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if len(argv) != 3 or argv[0] != "worker":
        raise SystemExit("usage: python -m aiko_services_amd.parallel.launch worker PLAN.json RANK")
    with open(argv[1]) as f:
        plan = Plan.from_json(f.read())
    rank = int(argv[2])
    if os.environ.get("AIKO_REJOIN_EPOCH"):
        rejoin(plan, rank)
        # no start barrier (the original group started long ago): the stage just serves
        pipeline = create_rank_pipeline(plan, rank, auto_start=False,
                                        extra_tags=[f"epoch={os.environ['AIKO_REJOIN_EPOCH']}"])
    else:
        join(plan, rank)
        pipeline = create_rank_pipeline(plan, rank)
    _watch_parent()
    if os.environ.get("AIKO_WORKER_SAMPLE"):             # sampled main-thread stacks -> DIR/worker_R.txt
        _sample_main_thread(os.path.join(os.environ["AIKO_WORKER_SAMPLE"], f"worker_{rank}.txt"))
    prof_dir = os.environ.get("AIKO_WORKER_PROFILE")      # cProfile of each worker's event loop
    if not prof_dir:
        pipeline.run(mqtt_connection_required=True)
        return
    import cProfile
    prof = cProfile.Profile()

    def dump():
        prof.disable()
        prof.dump_stats(os.path.join(prof_dir, f"worker_{rank}.prof"))
    atexit.register(dump)
    prof.enable()
    pipeline.run(mqtt_connection_required=True)


if __name__ == "__main__":
    worker_main()
