"""``aiko_pipeline`` command line (reference ``main/pipeline.py:1444-1555``).

    aiko_pipeline create DEFINITION [--name N] [--graph_path GP] [-p NAME VALUE]...
                  [--stream_id ID] [--stream_reset] [--grace_time S] [--show_response]
                  [--frame_id N] [--frame_data "(k: v ...)"] [--log_level L] [--log_mqtt M]
                  [--exit_after_frames N]
    aiko_pipeline destroy NAME

Also reachable as ``aiko pipeline create ...`` (:mod:`aiko_services_amd.tools.cli`).
``--exit_after_frames`` (new) terminates after N responses — for scripted runs and tests.
"""
from __future__ import annotations

import os
import queue
import sys
import threading

import click

from ..utils.configuration import get_pid


def describe(value):
    """Printable form of a response value: tensors (and DeviceResults, waited for) as dtype,
    shape and a SHA-256 prefix of their bytes — bit-exact comparisons across runs."""
    import hashlib
    try:
        import torch
    except ImportError:                                   # pragma: no cover
        torch = None
    if hasattr(value, "wait") and hasattr(value, "tensors"):
        return {k: describe(v) for k, v in value.wait().items()}
    if torch is not None and isinstance(value, torch.Tensor):
        t = value.detach().cpu().contiguous()
        digest = hashlib.sha256(t.view(torch.uint8).numpy().tobytes() if t.numel() else b"").hexdigest()[:16]
        return f"tensor({str(t.dtype).split('.')[-1]},{'x'.join(map(str, t.shape))},sha={digest})"
    if isinstance(value, dict):
        return {k: describe(v) for k, v in value.items()}
    return value


@click.group()
def main():
    """Create and destroy Pipelines"""


@main.command(help="Create Pipeline defined by PipelineDefinition pathname")
@click.argument("definition_pathname", nargs=1, type=str)
@click.option("--name", "-n", type=str, default=None, help="Pipeline name")
@click.option("--graph_path", "-gp", type=str, default=None,
              help="Pipeline Graph Path, use Head_PipelineElement_name")
@click.option("--parameters", "-p", type=click.Tuple((str, str)), default=None, multiple=True,
              help="Define Stream parameters")
@click.option("--stream_reset", "--reset", "-r", is_flag=True,
              help="Reset the remote Stream by invoking destroy_stream() first")
@click.option("--stream_id", "-s", type=str, default=None,
              help='Create Stream with identifier with optional process_id "name_{}"')
@click.option("--stream_parameters", "-sp", type=click.Tuple((str, str)), default=None, multiple=True,
              help="(deprecated) Define Stream parameters")
@click.option("--grace_time", "-gt", type=int, default=60, help="Stream receive frame time-out duration")
@click.option("--show_response", "-sr", is_flag=True, help="Show pipeline output response (output)")
@click.option("--frame_id", "-fi", type=int, default=0, help="Process Frame with identifier")
@click.option("--frame_data", "-fd", type=str, default=None, help="Process Frame with data")
@click.option("--log_level", "-ll", type=str, default="INFO", help="error, warning, info, debug")
@click.option("--log_mqtt", "-lm", type=str, default="all", help="all, false (console), true (mqtt)")
@click.option("--exit_after_frames", "-x", type=int, default=None,
              help="Terminate after this many frame responses")
def create(definition_pathname, graph_path, name, parameters, stream_id, stream_parameters, frame_id,
           frame_data, grace_time, show_response, log_level, log_mqtt, stream_reset, exit_after_frames):
    os.environ["AIKO_LOG_LEVEL"] = log_level.upper()
    os.environ["AIKO_LOG_MQTT"] = log_mqtt
    import logging
    for lg in logging.Logger.manager.loggerDict.values():   # apply to loggers created earlier too
        if isinstance(lg, logging.Logger):
            try:
                lg.setLevel(log_level.upper())
            except ValueError:
                pass
    from ..runtime.process import aiko
    from .definition import DefinitionError, parse_pipeline_definition
    from .engine import PipelineImpl, _LOGGER

    if stream_id:
        stream_id = stream_id.replace("{}", get_pid())
    if stream_parameters:
        _LOGGER.warning('"--stream_parameters" replaced by "--parameters"')
        parameters = stream_parameters
    if not os.path.exists(definition_pathname):
        raise SystemExit(f"Error: PipelineDefinition not found: {definition_pathname}")
    try:
        definition = parse_pipeline_definition(definition_pathname)
    except DefinitionError as exc:
        raise SystemExit(str(exc))

    response_queue = None
    if show_response or exit_after_frames:
        response_queue = queue.Queue()

        def response_handler(q):
            count = 0
            while True:
                info, data = q.get()
                count += 1
                if show_response:
                    _LOGGER.info(f"Output: <{info['stream_id']}:{info['frame_id']}> {describe(data)}")
                if exit_after_frames and count >= exit_after_frames:
                    aiko.process.terminate()
                    return
        threading.Thread(target=response_handler, args=(response_queue,), daemon=True).start()
        if stream_id is None and exit_after_frames:
            stream_id = "1"

    par = definition.parallel or {}
    staged = any(getattr(e.deploy, "stage", None) not in (None, 0) for e in definition.elements)
    if (par.get("mode", "pp") != "none" and int(par.get("gpus", 1)) > 1) or staged:
        # multi-GPU actor pipeline: one registered worker Pipeline per rank, hops over RCCL
        import json
        from ..parallel.launch import create_rank_pipeline, join, spawn_workers
        from ..parallel.placement import make_plan
        with open(definition_pathname) as f:
            plan = make_plan(json.load(f))
        if plan.mode == "dp":
            plan.stream = {"stream_id": stream_id or "1", "parameters": dict(parameters or {}),
                           "grace_time": grace_time}
            stream_id = stream_id or "1"
        _LOGGER.info(f"Parallel plan {plan.group}: stages {plan.stages} replicas {plan.replicas} "
                     f"local_share {plan.local_share}")
        spawn_workers(plan)
        join(plan, 0)
        pipeline = create_rank_pipeline(plan, 0, stream_id=stream_id, parameters=dict(parameters or {}),
                                        frame_id=frame_id, frame_data=frame_data, grace_time=grace_time,
                                        queue_response=response_queue, name=name, graph_path=graph_path,
                                        stream_reset=stream_reset, definition_pathname=definition_pathname)
        pipeline.run(mqtt_connection_required=True)
        return
    pipeline = PipelineImpl.create_pipeline(definition_pathname, definition, name, graph_path, stream_id,
                                            parameters, frame_id, frame_data, grace_time,
                                            queue_response=response_queue, stream_reset=stream_reset)
    pipeline.run(mqtt_connection_required=False)


@main.command(help="Destroy Pipeline")
@click.argument("name", nargs=1, type=str, required=True)
def destroy(name):
    from ..control.transport import ActorDiscovery, get_actor_mqtt
    from ..runtime import event
    from ..runtime.process import aiko
    from ..runtime.service import ServiceFilter
    from .engine import Pipeline

    def handler(command, details):
        if command == "add" and details:
            event.remove_timer_handler(waiting)
            get_actor_mqtt(f"{details[0]}/in", Pipeline).stop()
            print(f'Destroyed Pipeline "{name}"')
            aiko.process.terminate()

    def waiting():
        event.remove_timer_handler(waiting)
        print(f'Waiting to discover Pipeline "{name}"')

    ActorDiscovery(aiko.process).add_handler(handler, ServiceFilter("*", name, "*", "*", "*", "*"))
    event.add_timer_handler(waiting, 0.5)
    aiko.process.run()


if __name__ == "__main__":
    sys.exit(main())
