"""Dataflow engine: Pipeline, PipelineElement, PipelineRemote (reference ``main/pipeline.py``).

A :class:`PipelineImpl` is an Actor owning a DAG of elements built from a PipelineDefinition.
Frames enter through ``process_frame(stream_dict, frame_data)`` (posted by MQTT, by a frame
generator thread, or called directly by an embedding such as ``bench.py``) and run through
the graph path in topological order; each element's ``process_frame(stream, **inputs)``
returns ``(StreamEvent, outputs)`` and the outputs are merged into the frame's ``swag``.

Semantics kept from the reference: input selection by declared input names
with ``(from: to)`` mapping properties on graph edges; per-element metrics; DROP_FRAME /
STOP (graceful destroy) / ERROR (immediate destroy) handling; streams with a grace lease
extended per frame; the default stream ``"*"`` auto-created; thread-local "current stream";
remote elements pause the frame (``paused_pe_name``) and ``process_frame_response``
continues after it; output routed to ``queue_response``, ``topic_response`` or ``/out``;
4-level ``get_parameter`` precedence; ``set_parameter(s)``.

MI355X additions: swag values may be device tensors, handed between local elements by
reference (the data plane never touches MQTT); elements can declare a ``device`` in their
deploy block (``GpuPipelineElement`` binds it); ``frame.metrics`` optionally carries GPU
event timings (``AIKO_GPU_TIMING=1``); graph paths are cached.
"""
from __future__ import annotations

import os
import threading
import time
import traceback
from abc import abstractmethod
from collections import OrderedDict, deque
from typing import Tuple

from ..control.share import services_cache_create_singleton
from ..control.transport import get_actor_mqtt
from ..runtime import event
from ..runtime.actor import Actor, ActorTopic
from ..runtime.context import Interface, compose_instance, pipeline_args, pipeline_element_args
from ..runtime.lease import Lease
from ..runtime.process import aiko
from ..runtime.service import ServiceFilter, ServiceProtocol, ServiceTags
from ..parallel import hop_state as _hop     # torch-free: control-plane processes stay light
from ..utils import fault as _fault
from ..utils import trace as _trace
from ..utils.configuration import get_gpu_configuration
from ..utils.graph import Graph, Node
from ..utils.misc import load_module
from ..message.tensor_payload import encode_message
from ..utils.sexpr import generate, parse
from .definition import (PipelineDefinition, PipelineElementDeployLocal, PipelineElementDeployRemote,
                         parse_pipeline_definition)
from .stream import (DEFAULT_STREAM_ID, FIRST_FRAME_ID, Frame, Stream, StreamEvent, StreamEventName,
                     StreamState)

__all__ = ["Pipeline", "PipelineElement", "PipelineElementImpl", "PipelineImpl", "PipelineRemote",
           "PipelineGraph", "PROTOCOL_PIPELINE", "PROTOCOL_ELEMENT", "GRACE_TIME"]

_VERSION = 0
ACTOR_TYPE_PIPELINE = "pipeline"
ACTOR_TYPE_ELEMENT = "pipeline_element"
PROTOCOL_PIPELINE = f"{ServiceProtocol.AIKO}/{ACTOR_TYPE_PIPELINE}:{_VERSION}"
PROTOCOL_ELEMENT = f"{ServiceProtocol.AIKO}/{ACTOR_TYPE_ELEMENT}:{_VERSION}"
GRACE_TIME = 60
STATUS_UPDATE_PERIOD = 3.0
_GPU_TIMING = get_gpu_configuration().timing
_UNDECODED = object()          # _process_initialize: the message's hop tensors still to receive

_LOGGER = aiko.logger(__name__)


class PipelineError(SystemExit):
    pass


# ---- graph -----------------------------------------------------------------------------------

class PipelineGraph(Graph):
    def add_element(self, node: Node):
        self.add(node)
        node.predecessors = OrderedDict()

    @property
    def element_count(self):
        return len(self._graph)

    @classmethod
    def get_element(cls, node):
        element = node.element
        if isinstance(element, RemoteReplicas):
            return element, node.name, False, "ready" if element.members or element.awaiting else "absent"
        if type(element).__name__ == "ServiceRemoteProxy":
            return element, node.name, False, "ready"
        lifecycle = element.share["lifecycle"]
        local = element.is_local()
        name = node.name if isinstance(element, PipelineRemote) else type(element).__name__
        return element, name, local, lifecycle

    def validate(self, definition, head_node_name):
        """Link predecessors; warn about inputs no predecessor (or mapping) can provide."""
        for node in self.get_path(head_node_name):
            element, element_name, _, _ = PipelineGraph.get_element(node)
            for succ in node.successors:
                self.get_node(succ).predecessors[node.name] = node
        for node in self.get_path(head_node_name):
            if not node.predecessors:
                continue
            element = node.element
            definition_e = getattr(element, "definition", None)
            if definition_e is None:
                continue
            produced = set()
            stack = list(node.predecessors.values())
            seen = set()
            while stack:
                p = stack.pop()
                if p.name in seen:
                    continue
                seen.add(p.name)
                pd = getattr(p.element, "definition", None)
                if pd is not None:
                    produced.update(o["name"] for o in pd.output)
                stack.extend(p.predecessors.values())
            mapped = set()
            for mapping in definition.map_in_nodes.get(node.name, {}).values():
                mapped.update(mapping.values())
            for inp in definition_e.input:
                if inp["name"] not in produced and inp["name"] not in mapped:
                    _LOGGER.debug(f"PipelineElement {node.name}: input \"{inp['name']}\" "
                                  "not produced by any previous PipelineElement")


# ---- PipelineElement -----------------------------------------------------------------------

class PipelineElement(Actor):
    Interface.default("PipelineElement", "aiko_services_amd.pipeline.engine.PipelineElementImpl")

    @abstractmethod
    def create_frame(self, stream, frame_data):
        pass

    @abstractmethod
    def create_frames(self, stream, frame_generator, frame_id=FIRST_FRAME_ID, rate=None):
        pass

    @abstractmethod
    def get_parameter(self, name, default=None, use_pipeline=True):
        pass

    @abstractmethod
    def get_stream(self):
        pass

    @classmethod
    def is_local(cls):
        return True

    @abstractmethod
    def my_id(self, all=False):
        pass

    @abstractmethod
    def process_frame(self, stream, **kwargs) -> Tuple[int, dict]:
        pass

    @abstractmethod
    def start_stream(self, stream, stream_id):
        pass

    @abstractmethod
    def stop_stream(self, stream, stream_id):
        pass


class PipelineElementImpl(PipelineElement):
    def __init__(self, context):
        self.definition = context.get_definition()
        self.pipeline = context.get_pipeline()
        self.is_pipeline = self.pipeline is None
        if context.protocol == "*":
            context.set_protocol(PROTOCOL_PIPELINE if self.is_pipeline else PROTOCOL_ELEMENT)
        context.get_implementation("Actor").__init__(self, context)
        log_level, found = self.get_parameter("log_level", self_share_priority=False)
        if found:
            try:
                self.logger.setLevel(str(log_level).upper())
            except ValueError:
                pass
        self.share["source_file"] = f"v{_VERSION}⇒ {__file__}"
        params = getattr(self.definition, "parameters", None) or {}
        self.share.update(params)

    def create_frame(self, stream, frame_data, frame_id=None):
        frame_id = frame_id if frame_id is not None else stream.frame_id
        stream_copy = Stream(stream_id=stream.stream_id, frame_id=frame_id,
                             parameters=stream.parameters, queue_response=stream.queue_response,
                             state=stream.state, topic_response=stream.topic_response)
        self.pipeline.create_frame(stream_copy, frame_data)

    def create_frames(self, stream, frame_generator, frame_id=FIRST_FRAME_ID, rate=None):
        t = threading.Thread(target=self._create_frames_generator,
                             args=(stream, frame_generator, int(frame_id), rate), daemon=True,
                             name=f"frames-{self.name}")
        t.start()
        return t

    def _create_frames_generator(self, stream, frame_generator, frame_id, rate):
        pipeline = self.pipeline
        try:
            pipeline._enable_thread_local("_create_frames_generator", stream.stream_id, frame_id)
            stream, frame_id = self.get_stream()
            period = 1.0 / rate if rate else 0.0
            next_time = time.monotonic()
            while stream.state == StreamState.RUN:
                try:
                    stream_event, frame_data = frame_generator(stream, frame_id)
                except Exception:
                    self.logger.error("Exception in frame_generator()")
                    stream_event = StreamEvent.ERROR
                    frame_data = {"diagnostic": traceback.format_exc()}
                stream.state = pipeline._process_stream_event(self.name, stream_event, frame_data)
                if stream.state == StreamState.RUN and frame_data:
                    if isinstance(frame_data, dict):
                        frame_data = [frame_data]
                    if isinstance(frame_data, list):
                        for fd in frame_data:
                            # credit window: block THIS thread (never the actor's) while the
                            # pipeline has its limit of generated frames in flight
                            if not pipeline.admit_frame(stream.stream_id, frame_id):
                                stream.state = StreamState.ERROR
                                self.logger.error(f"frame generator: no frame completed for "
                                                  f"{pipeline.admission_timeout:g}s (window "
                                                  f"{pipeline.frame_window()}): stopping")
                                break
                            self.create_frame(stream, fd, frame_id)
                            frame_id += 1
                    else:
                        self.logger.warning("Frame generator must return either {frame_data} or [{frame_data}]")
                else:
                    frame_id += 1
                if stream.state in (StreamState.DROP_FRAME, StreamState.RUN):
                    stream.state = StreamState.RUN
                    if period:
                        next_time += period
                        delay = next_time - time.monotonic()
                        if delay > 0:
                            time.sleep(delay)
                        else:
                            next_time = time.monotonic()
                    pipeline.thread_local.frame_id = frame_id
        finally:
            pipeline._disable_thread_local("_create_frames_generator")

    def get_parameter(self, name, default=None, use_pipeline=True, self_share_priority=True):
        value, found = None, False
        definition = self.definition
        element_params = getattr(definition, "parameters", None) or {}
        stream_params = self._get_stream_parameters()
        qualified = f"{getattr(definition, 'name', self.name)}.{name}"
        if qualified in stream_params:
            value, found = stream_params[qualified], True
        elif name in element_params:
            value = self.share[name] if self_share_priority and name in self.share else element_params[name]
            found = True
        if not found and use_pipeline and not self.is_pipeline:
            if name in stream_params:
                value, found = stream_params[name], True
            else:
                pparams = getattr(self.pipeline.definition, "parameters", None) or {}
                if name in pparams:
                    value = (self.pipeline.share[name] if self_share_priority and name in self.pipeline.share
                             else pparams[name])
                    found = True
        if not found and default is not None:
            value = default
        return value, found

    def get_stream(self):
        return self.pipeline.get_stream()

    def _get_stream_parameters(self):
        try:
            stream, _ = self.get_stream()
            if stream:
                return stream.parameters
        except (AttributeError, AssertionError):
            pass
        return {}

    def my_id(self, all=False):
        name = self.name if all else ""
        try:
            stream, frame_id = self.get_stream()
            return f"{name}<{stream.stream_id}:{frame_id}>"
        except (AttributeError, AssertionError):
            return f"{name}<?>"

    def start_stream(self, stream, stream_id):
        return StreamEvent.OKAY, None

    def stop_stream(self, stream, stream_id):
        return StreamEvent.OKAY, None

    def process_frame(self, stream, **kwargs):
        return StreamEvent.OKAY, {}


# ---- Pipeline -------------------------------------------------------------------------------

class Pipeline(PipelineElement):
    Interface.default("Pipeline", "aiko_services_amd.pipeline.engine.PipelineImpl")

    @abstractmethod
    def create_stream(self, stream_id, graph_path=None, parameters=None, grace_time=GRACE_TIME,
                      queue_response=None, topic_response=None):
        pass

    @abstractmethod
    def destroy_stream(self, stream_id, graceful=False):
        pass

    @abstractmethod
    def process_frame_response(self, stream, frame_data):
        pass

    @abstractmethod
    def process_frames(self, stream_dicts, frame_datas):
        """Several frames in one message (a remote hop group, see ``parallel/hop.py``)."""

    @abstractmethod
    def process_frame_responses(self, stream_dicts, frame_datas):
        """The responses of several frames in one message."""

    @abstractmethod
    def set_parameter(self, stream_id, name, value):
        pass

    @abstractmethod
    def set_parameters(self, stream_id, parameters):
        pass


class PipelineImpl(Pipeline):
    def __init__(self, context):
        context.get_implementation("PipelineElement").__init__(self, context)
        self.share["definition_pathname"] = context.definition_pathname
        self.share["lifecycle"] = "waiting"
        self.share["graph_path"] = context.graph_path
        self.remote_pipelines: dict = {}
        self.services_cache = None
        self.stream_leases: dict = {}
        self.thread_local = threading.local()
        self.frames_completed = 0
        self._latencies: deque = deque(maxlen=1024)     # recent frame latencies (s) -> p50 / p99
        self.gpu_event_log: deque = deque(maxlen=4096)  # (element, start, end) HIP events (AIKO_GPU_TIMING)
        # remote hops: frames in flight per (stream_id, frame_id), frames waiting for a credit,
        # generator admission window (see dispatch / admit_frame below)
        self._inflight: dict = {}
        self._pending_hops: dict = {}      # remote node name -> FIFO of frames waiting for a credit
        self._admit_cv = threading.Condition()
        self._admitted: set = set()
        self._admit_deferred: set = set()   # credits handed to a Dropped send (released on its completion)
        self._window_limits: dict = {}
        self._hop_watch = False
        self.hops_failed = 0
        self.hops_redispatched = 0
        self.frames_dropped = 0
        self.hop_groups = 0                # group messages sent (hop_batch > 1)
        self._draining = False
        self._response_batch = None        # replica: responses of a group message, sent as one
        self._deferred_adds: dict = {}     # hop rank -> registrar add of a restarted replica
        self._readmit_hooked = False
        self.pipeline_graph = self._create_pipeline_graph(context.definition)
        self.share["element_count"] = self.pipeline_graph.element_count
        self.share["streams"] = 0
        self.share["streams_frames"] = 0
        self._update_lifecycle_state()
        event.add_timer_handler(self._status_update_timer, STATUS_UPDATE_PERIOD)

    # ---- lifecycle / status ------------------------------------------------------------------
    def _update_lifecycle_state(self):
        ready = all(PipelineGraph.get_element(n)[3] == "ready"
                    for n in self.pipeline_graph.get_path(self.share["graph_path"]))
        self.ec_producer.update("lifecycle", "ready" if ready else "waiting")

    def _status_update_timer(self):
        frames = sum(len(l.stream.frames) for l in self.stream_leases.values())
        self.ec_producer.update("streams", len(self.stream_leases))
        self.ec_producer.update("streams_frames", frames)
        self.ec_producer.update("frames_completed", self.frames_completed)
        stats = self.latency_stats()
        if stats:
            self.ec_producer.update("latency_p50_ms", stats["p50_ms"])
            self.ec_producer.update("latency_p99_ms", stats["p99_ms"])

    def latency_stats(self) -> dict:
        """p50 / p99 / max over the last 1024 completed frames (first element to last)."""
        lat = sorted(self._latencies)
        if not lat:
            return {}
        pick = lambda q: lat[min(len(lat) - 1, int(q * len(lat)))] * 1e3
        return {"frames": len(lat), "p50_ms": round(pick(0.50), 3), "p99_ms": round(pick(0.99), 3),
                "max_ms": round(lat[-1] * 1e3, 3)}

    def gpu_element_ms(self) -> dict:
        """Median GPU ms per frame of each local GPU element over the completed events in
        ``gpu_event_log`` (``AIKO_GPU_TIMING=1``; the placement balancer's input).  The median
        keeps first-frame tuning / graph capture out of the figure."""
        acc: dict = {}
        for name, start, end in list(self.gpu_event_log):
            if end is None or not end.query():
                continue
            acc.setdefault(name, []).append(start.elapsed_time(end))
        return {name: round(sorted(v)[len(v) // 2], 4) for name, v in acc.items() if v}

    def _add_node_properties(self, node_name, properties, predecessor_name):
        d = self.definition
        d.map_in_nodes.setdefault(node_name, {})[predecessor_name] = properties
        d.map_out_nodes.setdefault(predecessor_name, {})[node_name] = properties

    # ---- thread-local current stream ----------------------------------------------------------
    def _enable_thread_local(self, function_name, stream_id, frame_id=None):
        assert not getattr(self.thread_local, "stream", None), "thread_local.stream already assigned"
        self.thread_local.stream = self.stream_leases[stream_id].stream
        self.thread_local.frame_id = frame_id if frame_id is not None else self.thread_local.stream.frame_id

    def _disable_thread_local(self, function_name):
        self.thread_local.stream = None
        self.thread_local.frame_id = None

    def get_stream(self):
        stream = getattr(self.thread_local, "stream", None)
        assert stream, "thread_local.stream must be assigned"
        return stream, self.thread_local.frame_id

    def current_frame(self):
        """The Frame being processed on this thread (None outside ``process_frame``)."""
        stream = getattr(self.thread_local, "stream", None)
        if stream is None:
            return None
        return stream.frames.get(self.thread_local.frame_id)

    # ---- construction ----------------------------------------------------------------------------
    def create_frame(self, stream_dict, frame_data):
        if isinstance(stream_dict, Stream):
            stream_dict = stream_dict.as_dict()
        self._post_message(ActorTopic.IN, "process_frame", [stream_dict, frame_data])

    @classmethod
    def create_pipeline(cls, definition_pathname, pipeline_definition, name, graph_path, stream_id,
                        parameters, frame_id, frame_data, grace_time, queue_response=None,
                        stream_reset=False, tags=None):
        name = name or pipeline_definition.name
        init_args = pipeline_args(name, protocol=PROTOCOL_PIPELINE, definition=pipeline_definition,
                                  definition_pathname=definition_pathname, graph_path=graph_path,
                                  tags=tags)
        pipeline = compose_instance(PipelineImpl, init_args)
        stream_dict = {"frame_id": int(frame_id or 0), "parameters": {}}
        parameters = dict(parameters or {})
        if stream_id is not None:
            stream_dict["stream_id"] = stream_id
            if stream_reset:
                pipeline.destroy_stream(stream_id)
            pipeline.create_stream(stream_id, graph_path=None, parameters=parameters,
                                   grace_time=grace_time, queue_response=queue_response)
        else:
            pipeline.set_parameters(None, list(parameters.items()))
        if frame_data is not None:
            _, arguments = parse(f"(process_frame {frame_data})")
            if not arguments:
                raise SystemExit("Error: Frame data must be provided")
            pipeline.create_frame(stream_dict, arguments[0])
        return pipeline

    def _error_pipeline(self, header, diagnostic):
        PipelineImpl._exit(header, diagnostic)

    @classmethod
    def _exit(cls, header, diagnostic):
        _LOGGER.error(f"{header}\n{diagnostic}")
        raise PipelineError(-1)

    def _load_element_class(self, module_descriptor, class_name, header):
        try:
            module = load_module(module_descriptor)
            return getattr(module, class_name)
        except FileNotFoundError:
            self._error_pipeline(header, f"PipelineDefinition: PipelineElement {class_name}: "
                                 f"Module {module_descriptor} could not be found")
        except Exception:
            self._error_pipeline(header, f"PipelineDefinition: PipelineElement {class_name}: "
                                 f"Module {module_descriptor} could not be loaded\n{traceback.format_exc()}")

    def _create_pipeline_graph(self, definition: PipelineDefinition):
        header = f"Error: Creating Pipeline: {definition.name}"
        if not definition.elements:
            self._error_pipeline(header, "PipelineDefinition: Doesn't define any PipelineElements")
        definition.map_in_nodes = {}
        definition.map_out_nodes = {}
        heads, successors = Graph.traverse(definition.graph, self._add_node_properties)
        graph = PipelineGraph(heads)
        for ed in definition.elements:
            if ed.name not in successors:
                _LOGGER.debug(f"Skipping PipelineElement {ed.name}: not used within the graph")
                continue
            deploy = ed.deploy
            if isinstance(deploy, PipelineElementDeployLocal):
                element_class = self._load_element_class(deploy.module, deploy.class_name, header)
            elif isinstance(deploy, PipelineElementDeployRemote):
                element_class = PipelineRemote
            else:
                self._error_pipeline(header, f"PipelineElement type unknown: {type(deploy).__name__}")
            init_args = pipeline_element_args(ed.name, definition=ed, pipeline=self)
            instance = compose_instance(element_class, init_args)
            instance.parameters = ed.parameters
            if element_class is PipelineRemote:
                service_name = deploy.service_filter["name"]
                if service_name in self.remote_pipelines:
                    self._error_pipeline(header, f"PipelineElement {ed.name}: re-uses remote service_filter "
                                         f"name: {service_name}")
                self.remote_pipelines[service_name] = (ed.name, instance, None)
                if self.services_cache is None:
                    self.services_cache = services_cache_create_singleton(self)
                self.services_cache.add_handler(self._pipeline_element_change_handler,
                                                ServiceFilter.with_topic_path(**deploy.service_filter))
            graph.add_element(Node(ed.name, instance, successors[ed.name]))
        missing = [n for n in successors if n not in graph._graph]
        if missing:
            self._error_pipeline(header, f"PipelineDefinition: graph references undefined "
                                 f"PipelineElements: {', '.join(missing)}")
        graph.validate(definition, self.share["graph_path"])
        return graph

    def _pipeline_element_change_handler(self, command, service_details):
        """Registrar add/remove of a service matching a remote element's filter.  Every
        matching service becomes a member of the element's :class:`RemoteReplicas` (one for
        the reference's single remote Pipeline; several when a stage is replicated).  A
        ``rank=N`` tag marks a service reachable on the RCCL data plane (``parallel/hop.py``)."""
        if command not in ("add", "remove") or not service_details:
            return
        topic_path = f"{service_details[0]}/in"
        service_name = service_details[1]
        if service_name not in self.remote_pipelines:
            return
        element_name, element_instance, replicas = self.remote_pipelines[service_name]
        node = self.pipeline_graph.get_node(element_name)
        if replicas is None:
            replicas = RemoteReplicas(element_instance.definition)
        if command == "add":
            tags = ServiceTags.parse_tags(service_details[5] if len(service_details) > 5
                                          and isinstance(service_details[5], list) else [])
            rank = tags.get("rank")
            hop = _hop.plane()
            if hop is not None and rank not in (None, "") and hop.is_dead(int(rank)):
                # a restarted replica on a rank whose links were retired: it stays absent until
                # its fresh links are up (parallel/launch.py rejoin), then this add runs again
                self._deferred_adds[int(rank)] = (command, service_details)
                if not self._readmit_hooked:
                    hop.on_readmit(lambda peer: self._post_message(
                        ActorTopic.IN, "hop_readmitted", [peer], target_function=self._hop_readmitted))
                    self._readmit_hooked = True
                self.logger.info(f"remote {element_name}: rank {rank} re-registered "
                                 f"(epoch {tags.get('epoch', '?')}): waiting for its data-plane links")
                return
            proxy = get_actor_mqtt(topic_path, PipelineRemote)
            proxy.definition = element_instance.definition
            proxy.hop_rank = int(rank) if rank not in (None, "") else None
            replicas.add(topic_path, proxy, weight=float(tags.get("weight", 1) or 1))
            element_instance.set_remote_absent(False)
            # a member that appears while streams run (a restarted replica, a late registrar add)
            # gets each of them first: on its topic the create_stream precedes any frame
            for sid, lease in list(self.stream_leases.items()):
                st = lease.stream
                on_path = any(PipelineGraph.get_element(n)[1] == element_name
                              for n in self.pipeline_graph.get_path(Graph.path_local(st.graph_path)))
                if on_path:
                    proxy.create_stream(sid, Graph.path_remote(st.graph_path), st.parameters,
                                        getattr(lease, "grace_time", GRACE_TIME), None, self.topic_in)
        else:
            if topic_path not in replicas._members:
                return
            self.remote_pipelines[service_name] = (element_name, element_instance, replicas)
            self._replica_lost(service_name, topic_path)
            return
        self.remote_pipelines[service_name] = (element_name, element_instance, replicas)
        if replicas.members:
            node.element = replicas
        else:
            element_instance.set_remote_absent(True)
            node.element = element_instance
        self._update_lifecycle_state()

    def _hop_readmitted(self, rank):
        """A restarted peer's hop links are up again: its deferred registrar add now binds it."""
        pending = self._deferred_adds.pop(int(rank), None)
        if pending is not None:
            self.logger.info(f"hop rank {rank} re-admitted: replica bound again")
            self._pipeline_element_change_handler(*pending)
            if self._pending_hops:
                self._drain_pending()

    # ---- streams -------------------------------------------------------------------------------
    def create_stream(self, stream_id, graph_path=None, parameters=None, grace_time=GRACE_TIME,
                      queue_response=None, topic_response=None):
        if queue_response and topic_response:
            self.logger.error("Create stream: use either queue_response or topic_response")
            return False
        if self.share["lifecycle"] != "ready":
            self._post_message(ActorTopic.IN, "create_stream",
                               [stream_id, graph_path, parameters, grace_time, queue_response, topic_response],
                               delay=1.0)
            self.logger.warning(f"Create stream: {stream_id}: remote Pipeline not yet discovered ... will retry")
            return False
        stream_id = str(stream_id)
        if stream_id in self.stream_leases:
            if topic_response is not None:
                # another upstream replica (or a restarted one) opening the same stream: its
                # frames carry their own reply topic (``reply_to``), nothing to do
                self.logger.info(f"Create stream: {stream_id} already exists (upstream {topic_response})")
            else:
                self.logger.error(f"Create stream: {stream_id} already exists")
            return False
        graph_path = graph_path or self.share["graph_path"]
        if graph_path and Graph.path_local(graph_path) not in self.pipeline_graph.head_nodes:
            self.logger.error(f"Create stream: Unknown Pipeline Graph Path: {graph_path}")
            return False
        lease = Lease(int(float(grace_time)), stream_id, lease_expired_handler=self.destroy_stream)
        lease.grace_time = grace_time
        lease.stream = Stream(stream_id=stream_id, graph_path=graph_path,
                              parameters=parameters if isinstance(parameters, dict) else {},
                              queue_response=queue_response, topic_response=topic_response)
        self.stream_leases[stream_id] = lease
        try:
            self._enable_thread_local("create_stream", stream_id)
            stream, _ = self.get_stream()
            for node in self.pipeline_graph.get_path(Graph.path_local(stream.graph_path)):
                element, element_name, local, _ = PipelineGraph.get_element(node)
                if local:
                    try:
                        stream_event, diagnostic = element.start_stream(stream, stream_id)
                    except Exception:
                        self.logger.error("Exception in pipeline.create_stream() --> start_stream()")
                        stream_event, diagnostic = StreamEvent.ERROR, {"diagnostic": traceback.format_exc()}
                    self._process_stream_event(element_name, stream_event, diagnostic)
                    if stream_id not in self.stream_leases:
                        break   # start_stream failed -> stream destroyed
                else:
                    element.create_stream(stream_id, Graph.path_remote(stream.graph_path), parameters,
                                          grace_time, None, self.topic_in)
        finally:
            self._disable_thread_local("create_stream")
        return True

    def destroy_stream(self, stream_id, graceful=False, use_thread_local=True):
        stream_id = str(stream_id)
        if isinstance(graceful, str):
            graceful = graceful.lower() == "true"
        lease = self.stream_leases.get(stream_id)
        if graceful and lease is not None and lease.stream.frames:
            # drain first, THEN tell the remote elements: the reference
            # (/root/reference/src/aiko_services/main/pipeline.py:804-809) destroys the remote
            # stream before its own frames — some still to be forwarded — have drained, so a
            # downstream stage can drop the tail of a stream ("stream not found")
            self._post_message(ActorTopic.IN, "destroy_stream", [stream_id, graceful, use_thread_local],
                               delay=0.05 if self._inflight or self._pending_total() else 1.0)
            return False
        if self.share["lifecycle"] == "ready":
            for node in self.pipeline_graph.get_path(self.share["graph_path"]):
                element, _, local, _ = PipelineGraph.get_element(node)
                if not local:
                    element.destroy_stream(stream_id, True)
        else:
            self._post_message(ActorTopic.IN, "destroy_stream", [stream_id, graceful, use_thread_local],
                               delay=1.0)
            return False
        lease = self.stream_leases.get(stream_id)
        if lease is None:
            return False
        enabled = False
        try:
            if use_thread_local and not getattr(self.thread_local, "stream", None):
                self._enable_thread_local("destroy_stream", stream_id)
                enabled = True
            stream = lease.stream
            if graceful and stream.frames:
                self._post_message(ActorTopic.IN, "destroy_stream", [stream_id, graceful, use_thread_local],
                                   delay=1.0)
                return False
            for node in self.pipeline_graph.get_path(Graph.path_local(stream.graph_path)):
                element, element_name, local, _ = PipelineGraph.get_element(node)
                if local:
                    try:
                        stream_event, diagnostic = element.stop_stream(stream, stream_id)
                    except Exception:
                        self.logger.error("Exception in pipeline.destroy_stream() --> stop_stream()")
                        stream_event, diagnostic = StreamEvent.ERROR, {"diagnostic": traceback.format_exc()}
                    self._process_stream_event(element_name, stream_event, diagnostic, in_destroy_stream=True)
        finally:
            if enabled:
                self._disable_thread_local("destroy_stream")
        lease = self.stream_leases.pop(stream_id, None)
        if lease is not None:
            lease.terminate()
            lease.stream.state = StreamState.STOP if lease.stream.state != StreamState.ERROR else StreamState.ERROR
            # frames still in flight (a non-graceful destroy, or an error) leave with the stream:
            # their hop / FramePool slots and admission credits come back now — a response that
            # arrives later finds "stream not found" and is dropped.  A frame still out on a
            # remote hop is dropped first: a zero-copy send keeps its producer slot until the
            # transfer has completed (hop.drop), a queued one simply leaves its queue.
            hop = _hop.plane()
            pending = {}
            for key in [k for k in self._inflight if str(k[0]) == stream_id]:
                f = self._inflight.pop(key)
                if hop is not None and f["rank"] is not None:
                    pending[key[1]] = hop.drop(key)
            for node_name, fifo in list(self._pending_hops.items()):
                for p in [p for p in fifo if str(p["stream_id"]) == stream_id]:
                    fifo.remove(p)
                    if p["held"] and hop is not None:
                        pending[p["frame_id"]] = hop.drop((p["stream_id"], p["frame_id"]))
            for frame_id in list(lease.stream.frames):
                self._release_frame(lease.stream, frame_id, after=pending.get(frame_id))
        self._admit_release_stream(stream_id)
        hop = _hop.plane()
        if hop is not None:
            self.logger.info(f"Stream {stream_id} destroyed: hop {hop.stats()} redispatched "
                             f"{self.hops_redispatched} failed {self.hops_failed} dropped {self.frames_dropped}")
        return True

    # ---- frames ----------------------------------------------------------------------------------
    def process_frame(self, stream_dict, frame_data):
        return self._process_frame_common(stream_dict, frame_data, True)

    def process_frame_response(self, stream_dict, frame_data):
        return self._process_frame_common(stream_dict, frame_data, False)

    # ---- hop groups: several frames per control message + transfer -----------------------------
    def process_frames(self, stream_dicts, frame_datas):
        return self._process_group(stream_dicts, frame_datas, True)

    def process_frame_responses(self, stream_dicts, frame_datas):
        return self._process_group(stream_dicts, frame_datas, False)

    def _process_group(self, stream_dicts, frame_datas, new_frame):
        """A group message (``hop_batch`` > 1 at the sender): ONE receive for every member's
        tensors, then each member runs as its own frame.  A replica answers the members that
        complete here with ONE ``process_frame_responses`` per reply rank."""
        if not isinstance(stream_dicts, list) or not isinstance(frame_datas, list) \
                or len(stream_dicts) != len(frame_datas):
            self.logger.warning("Process frames: stream dicts and frame data must be lists of one length")
            return False
        frame_datas = [d if isinstance(d, dict) else {} for d in frame_datas]
        hop = _hop.plane()
        if hop is None:
            for sd, fd in zip(stream_dicts, frame_datas):
                self._process_frame_common(sd, fd, new_frame)
            return True
        try:
            outs, handle, work = hop.decode_group_async(frame_datas, pooled=new_frame)
            if work is not None:
                if hop.host_transfers:
                    hop.finish_later(work, lambda error: self._post_message(
                        ActorTopic.IN, "hop_group_arrived", [stream_dicts, outs, handle, work, new_frame, error],
                        target_function=self._hop_group_arrived))
                    return True
                hop.finish(work, handle)
        except _hop.StageFailure as exc:
            self.logger.error(f"Process frames: {exc}")
            self._replica_lost_rank(exc.peer)
            return False
        return self._group_continue(stream_dicts, outs, handle, new_frame)

    def _hop_group_arrived(self, stream_dicts, outs, handle, work, new_frame, error):
        try:
            _hop.plane().complete(work, handle, error)
        except _hop.StageFailure as exc:
            self.logger.error(f"Process frames: {exc}")
            self._replica_lost_rank(exc.peer)
            return False
        return self._group_continue(stream_dicts, outs, handle, new_frame)

    def _group_continue(self, stream_dicts, outs, handle, new_frame):
        outer = self._response_batch
        batch = self._response_batch = [] if outer is None else outer
        try:
            for sd, values in zip(stream_dicts, outs):
                self._process_frame_common(sd, values, new_frame, decoded=handle)
        finally:
            if batch is not outer:
                self._response_batch = outer
                self._flush_responses(batch)
        return True

    def _flush_responses(self, batch):
        """Send the responses collected while a group ran: one message + one transfer per
        (response topic, reply rank), then release their frames (after the staging copies, so
        no receive slot is reused under them)."""
        hop = _hop.plane()
        groups: dict = {}
        for topic, reply, info, data, ready, stream, frame_id in batch:
            groups.setdefault((topic, reply), []).append((info, data, ready))
        try:
            # this runs after the members' lane scopes closed: every member's response is
            # ordered after the event recorded on its own lane when it completed
            for (topic, reply), items in groups.items():
                proxy = get_actor_mqtt(topic, Pipeline)
                if len(items) == 1:
                    proxy.process_frame_response(items[0][0], hop.encode(reply, items[0][1], ready=[items[0][2]]))
                else:
                    outs = hop.encode_group(reply, [data for _, data, _ in items], ready=[r for *_, r in items])
                    proxy.process_frame_responses([info for info, _, _ in items], outs)
        finally:
            for *_, stream, frame_id in batch:
                self._release_frame(stream, frame_id)

    def _hop_arrived(self, stream_dict, values, handle, work, new_frame, error):
        """The bytes of a host-transfer hop message (gloo) arrived: resume its frame."""
        try:
            _hop.plane().complete(work, handle, error)
        except _hop.StageFailure as exc:
            self.logger.error(f"Process frame <{stream_dict.get('stream_id')}:{stream_dict.get('frame_id')}>: {exc}")
            self._replica_lost_rank(exc.peer)
            return False
        return self._process_frame_common(stream_dict, values, new_frame, decoded=handle)

    def _process_initialize(self, stream_dict, frame_data_in, new_frame, decoded=_UNDECODED):
        stream = Stream()
        if not stream.update(stream_dict):
            self.logger.warning("Process frame: stream_dict must be a dictionary")
            return None, None, None
        if frame_data_in == [] or frame_data_in is None:
            frame_data_in = {}
        if not isinstance(frame_data_in, dict):
            self.logger.warning("Process frame: frame data must be a dictionary")
            return None, None, None
        hop_handle = None
        hop = _hop.plane()
        if decoded is not _UNDECODED:
            hop_handle = decoded                 # resumed by _hop_arrived: the bytes are in
        elif hop is not None and _hop.needs_decode(stream_dict, frame_data_in):
            # tensors of this message arrive over RCCL: always receive them (even if the frame is
            # then rejected) so the link stays in order; forward hops land in FramePool slots
            try:
                if hop.host_transfers:
                    # gloo: the receive blocks the host until the bytes are in — wait on the
                    # plane's waiter thread and resume the frame from the mailbox, so the
                    # receives of several messages overlap (they are still POSTED in order)
                    values, handle, work = hop.decode_async(frame_data_in, pooled=new_frame)
                    if work is not None:
                        hop.finish_later(work, lambda error: self._post_message(
                            ActorTopic.IN, "hop_arrived", [stream_dict, values, handle, work, new_frame, error],
                            target_function=self._hop_arrived))
                        return None, None, None
                    frame_data_in, hop_handle = values, handle
                else:
                    frame_data_in, hop_handle = hop.decode(frame_data_in, pooled=new_frame)
            except _hop.StageFailure as exc:
                # the sender died mid-transfer: a response is re-dispatched (the frame is still
                # held, in flight toward that member) with every other frame the member held
                self.logger.error(f"Process frame <{stream.stream_id}:{stream.frame_id}>: {exc}")
                self._replica_lost_rank(exc.peer)
                return None, None, None
        if not new_frame:
            # the response of a remote hop: its credit (and held retransmit slot) is free again
            if hop is not None and stream_dict.get("hop_rank") is not None:
                hop.mark_alive(int(stream_dict["hop_rank"]))
            self._remote_done((stream.stream_id, stream.frame_id))
        graph, stream = self._process_initialize_stream(stream, stream_dict, frame_data_in, new_frame)
        if graph is None:
            if hop_handle is not None:
                hop.release([hop_handle])
            return None, None, None
        frame = stream.frames[stream.frame_id]
        if new_frame:
            frame.lane = getattr(self, "_frame_lane", None) if self._frame_lanes()[0] > 1 else None
        if hop_handle is not None:
            frame.hop_handles.append(hop_handle)
        if new_frame and stream_dict.get("hop_rank") is not None:
            frame.hop_reply = int(stream_dict["hop_rank"])
        if new_frame and stream_dict.get("reply_to"):
            frame.reply_to = str(stream_dict["reply_to"])
        return graph, stream, frame_data_in

    def _process_initialize_stream(self, stream, stream_dict, frame_data_in, new_frame):
        stream_id = stream.stream_id
        if stream_id == DEFAULT_STREAM_ID and DEFAULT_STREAM_ID not in self.stream_leases:
            if not self.create_stream(DEFAULT_STREAM_ID, graph_path=stream.graph_path,
                                      parameters=stream.parameters):
                return None, None
        frame_id = stream.frame_id
        header = f"Process frame <{stream_id}:{frame_id}>:"
        lease = self.stream_leases.get(stream_id)
        if lease is None:
            self.logger.warning(f"{header} stream not found")
            if new_frame:
                self._admit_release((stream_id, frame_id))   # admitted, but it never existed
                self._reject_remote(stream_dict, "stream not found")
            return None, None
        lease.extend()
        stream = lease.stream
        stream.frame_id = frame_id
        stream.state = int(stream_dict.get("state", StreamState.RUN)) if stream.state != StreamState.ERROR \
            else StreamState.ERROR
        graph = None
        if new_frame:
            if frame_id in stream.frames:
                self.logger.warning(f"{header} new frame id already exists")
                return None, None
            frame = stream.frames[frame_id] = Frame()
            graph = self.pipeline_graph.get_path(Graph.path_local(stream.graph_path))
        elif frame_id in stream.frames:
            frame = stream.frames[frame_id]
            graph = self.pipeline_graph.iterate_after(frame.paused_pe_name, Graph.path_local(stream.graph_path))
        else:
            self.logger.warning(f"{header} paused frame id doesn't exist")
            return None, None
        frame.swag.update(frame_data_in)
        return graph, stream

    def _reject_remote(self, stream_dict, diagnostic):
        """A frame sent by an upstream stage cannot run here (its stream is gone — e.g. this
        process was stopped while the sender timed the frame out and destroyed the stream):
        answer it with an ERROR response so the sender is not left waiting, and so it hears
        from this rank (its proof of life, ``HopPlane.mark_alive``)."""
        reply_to = stream_dict.get("reply_to") if isinstance(stream_dict, dict) else None
        if not reply_to:
            return
        info = {"stream_id": stream_dict.get("stream_id"), "frame_id": stream_dict.get("frame_id"),
                "state": StreamState.ERROR}
        hop = _hop.plane()
        if hop is not None:
            info["hop_rank"] = hop.rank
        get_actor_mqtt(str(reply_to), Pipeline).process_frame_response(info, {"diagnostic": diagnostic})

    def _frame_lanes(self):
        """(lanes, device) for ``gpu_lanes`` (see ``gpu/lanes.py``); decided on first use."""
        cached = getattr(self, "_lanes_cfg", None)
        if cached is not None:
            return cached
        lanes, found = self.get_parameter("gpu_lanes")
        if not found:
            lanes = os.environ.get("AIKO_GPU_LANES", 1)
        try:
            lanes = max(1, int(lanes))
        except (TypeError, ValueError):
            lanes = 1
        device = None
        if lanes > 1:
            for node in self.pipeline_graph:
                element, name, local, _ = PipelineGraph.get_element(node)
                if not local:
                    # a remote element ends the local part of the frame; its response resumes the
                    # frame on the lane it started on (Frame.lane)
                    continue
                if hasattr(element, "device") and hasattr(element, "run_maybe_captured"):
                    if not getattr(element, "lane_safe", False):
                        raise ValueError(f"gpu_lanes > 1: GPU element {name} is not lane-safe")
                    device = device or element.device
            if device is None or getattr(device, "type", "cpu") != "cuda":
                lanes = 1
        self._lanes_cfg = (lanes, device)
        self._lane_next = 0
        self.share["gpu_lanes"] = lanes
        return self._lanes_cfg

    def _process_frame_common(self, stream_dict, frame_data_in, new_frame, decoded=_UNDECODED):
        lanes, device = self._frame_lanes()
        if lanes > 1:
            from ..gpu.lanes import in_lane, lane_scope
            if in_lane():
                # nested pipeline (rank 0's local share of a replicated stage): the frame keeps
                # the lane of the enclosing frame
                return self._process_frame_body(stream_dict, frame_data_in, new_frame, decoded)
            lane = None
            if not new_frame:
                # a remote hop's response resumes the frame on the lane it started on
                lease = self.stream_leases.get(str(stream_dict.get("stream_id"))) \
                    if isinstance(stream_dict, dict) else None
                try:
                    frame = lease.stream.frames.get(int(stream_dict.get("frame_id"))) if lease else None
                except (TypeError, ValueError):
                    frame = None
                lane = getattr(frame, "lane", None)
            if lane is None:
                lane = self._lane_next
                self._lane_next = (lane + 1) % lanes
            self._frame_lane = lane
            with lane_scope(lane, device):
                return self._process_frame_body(stream_dict, frame_data_in, new_frame, decoded)
        return self._process_frame_body(stream_dict, frame_data_in, new_frame, decoded)

    def _process_frame_body(self, stream_dict, frame_data_in, new_frame, decoded=_UNDECODED):
        graph, stream, frame_data_in = self._process_initialize(stream_dict, frame_data_in, new_frame, decoded)
        if graph is None:
            return False
        frame_complete = True
        frame_id = stream.frame_id
        try:
            self._enable_thread_local("process_frame", stream.stream_id)
            frame = stream.frames[frame_id]
            metrics = frame.metrics
            if not metrics:
                metrics["pipeline_elements"] = {}
                metrics["time_pipeline_start"] = time.time()
                metrics["perf_pipeline_start"] = time.perf_counter()   # trace spans: one clock
            tracer = _trace.get_tracer()
            faults = _fault.active()
            frame_data_out = {} if new_frame else frame_data_in
            definition_pathname = self.share["definition_pathname"]
            for node in graph:
                if stream.state in (StreamState.DROP_FRAME, StreamState.ERROR):
                    break
                element, element_name, local, _ = PipelineGraph.get_element(node)
                header = (f'Error: Invoking Pipeline "{definition_pathname}": '
                          f'PipelineElement "{element_name}": process_frame()')
                inputs = self._process_map_in(header, element, node.name, frame.swag)
                target = None
                if isinstance(element, RemoteReplicas) and self.share["lifecycle"] == "ready":
                    target = element.pick(self._has_credit)
                    if isinstance(target, LocalStage):
                        # this frame's share of a replicated stage runs in-process (no hop)
                        stream_event, frame_data_out = target.run(stream.stream_id, frame_id, inputs)
                        stream.state = self._process_stream_event(element_name, stream_event, frame_data_out)
                        self._process_map_out(node.name, frame_data_out)
                        frame.swag.update(frame_data_out)
                        continue
                if local:
                    start = time.time()
                    p_start = time.perf_counter() if tracer is not None else 0.0
                    enter = getattr(element, "stream_enter", None)
                    hip_ctx = enter(frame) if enter is not None else None
                    gpu_t = element.gpu_timer_start() if (_GPU_TIMING or tracer is not None) \
                        and hasattr(element, "gpu_timer_start") else None
                    try:
                        if faults is not None:
                            faults.before_element(element_name, frame_id)
                        stream_event, frame_data_out = element.process_frame(stream, **inputs)
                    except Exception:
                        self.logger.error("Exception in pipeline.process_frame() --> element.process_frame()")
                        stream_event = StreamEvent.ERROR
                        frame_data_out = {"diagnostic": traceback.format_exc()}
                    if frame_data_out is None:
                        frame_data_out = {}
                    gpu_end = element.gpu_timer_stop(gpu_t) if gpu_t is not None else None
                    if enter is not None:
                        element.stream_exit(frame, frame_data_out, hip_ctx)
                    stream.state = self._process_stream_event(element_name, stream_event, frame_data_out)
                    self._process_map_out(node.name, frame_data_out)
                    t = time.time()
                    metrics["pipeline_elements"][f"time_{element.name}"] = t - start
                    metrics["time_pipeline"] = t - metrics["time_pipeline_start"]
                    if gpu_t is not None:
                        metrics.setdefault("gpu_events", {})[element.name] = gpu_t
                        self.gpu_event_log.append((element.name, gpu_t, gpu_end))
                        if tracer is not None:
                            tracer.gpu_span(element_name, gpu_t, gpu_end,
                                            args={"frame_id": frame_id},
                                            stream_name=getattr(element, "hip_stream_name", None) or "default")
                    if tracer is not None:
                        tracer.span(element_name, p_start, time.perf_counter(),
                                    args={"stream_id": stream.stream_id, "frame_id": frame_id})
                    hook = getattr(element, "frame_done", None)
                    if hook is not None:
                        hook(t - start)
                    frame.swag.update(frame_data_out)
                else:
                    if self.share["lifecycle"] != "ready":
                        stream.state = self._process_stream_event(
                            element_name, StreamEvent.ERROR,
                            {"diagnostic": "process_frame() invoked when remote Pipeline hasn't been discovered"})
                    else:
                        frame_complete = False
                        frame_data_out = {}
                        frame.paused_pe_name = node.name
                        if not isinstance(element, RemoteReplicas):
                            target = element
                        if target is None:
                            # no replica has a credit left: the frame waits (bounded queue)
                            self._queue_hop(element, node.name, stream.stream_id, frame_id, inputs)
                        else:
                            self._dispatch(element, target, node.name, stream.stream_id, frame_id, inputs)
                    break
            if frame_complete:
                join = getattr(stream.frames.get(frame_id), "_hip_join", None)
                if join is not None:
                    join()
                self.frames_completed += 1
                latency = time.time() - metrics["time_pipeline_start"]
                self._latencies.append(latency)
                if faults is not None:
                    faults.frame_completed()
                if tracer is not None:
                    end = time.perf_counter()
                    tracer.span(f"frame {self.name}", metrics.get("perf_pipeline_start", end - latency), end, cat="frame",
                                args={"stream_id": stream.stream_id, "frame_id": frame_id})
                stream_info = {"stream_id": stream.stream_id, "frame_id": frame_id, "state": stream.state}
                if stream.queue_response is not None:
                    if getattr(self, "response_swag", False):   # pipeline-parallel stage hand-off
                        frame_data_out = dict(frame.swag)
                    stream.queue_response.put((stream_info, frame_data_out))
                elif stream.topic_response or getattr(stream.frames.get(frame_id), "reply_to", None):
                    hop = _hop.plane()
                    done = stream.frames.get(frame_id)
                    reply = getattr(done, "hop_reply", None)
                    # the sender of THIS frame (a stage fed by several upstream replicas, or by a
                    # restarted one, answers each frame to its own sender)
                    topic = getattr(done, "reply_to", None) or stream.topic_response
                    if hop is not None and reply is not None and self._response_batch is not None:
                        # member of a group message: answered with the group, released after
                        stream_info["hop_rank"] = hop.rank
                        self._response_batch.append((topic, reply, stream_info, frame_data_out,
                                                     hop.ready_event(), stream, frame_id))
                        frame_complete = False
                    else:
                        if hop is not None and reply is not None:
                            frame_data_out = hop.encode(reply, frame_data_out)
                            stream_info["hop_rank"] = hop.rank     # the responder (proof of life)
                        get_actor_mqtt(topic, Pipeline).process_frame_response(stream_info, frame_data_out)
                else:
                    aiko.message.publish(self.topic_out, encode_message("process_frame", (stream_info, frame_data_out)))
        finally:
            if frame_complete:
                self._release_frame(stream, frame_id)
            self._disable_thread_local("process_frame")
            if stream.state == StreamState.DROP_FRAME:
                stream.state = StreamState.RUN
        return True

    def _process_map_in(self, header, element, node_name, swag):
        map_in = {}
        for mapping in self.definition.map_in_nodes.get(node_name, {}).values():
            if mapping:
                _from, to = next(iter(mapping.items()))
                map_in[to] = f"{node_name}.{to}"
        inputs = {}
        definition = getattr(element, "definition", None)
        for inp in (definition.input if definition is not None else []):
            name = inp["name"]
            key = map_in.get(name, name)
            if key in swag:
                inputs[name] = swag[key]
            elif name in swag:
                inputs[name] = swag[name]
            else:
                self._error_pipeline(header, f'Function parameter "{name}" not found')
        return inputs

    def _process_map_out(self, node_name, frame_data_out):
        for out_element, mapping in self.definition.map_out_nodes.get(node_name, {}).items():
            if mapping:
                from_name, to_name = next(iter(mapping.items()))
                if from_name in frame_data_out:
                    frame_data_out[f"{out_element}.{to_name}"] = frame_data_out.pop(from_name)

    def _process_stream_event(self, element_name, stream_event, diagnostic, in_destroy_stream=False):
        def get_diagnostic():
            name = StreamEventName.get(stream_event, str(stream_event))
            d = diagnostic.get("diagnostic", "No diagnostic provided") if isinstance(diagnostic, dict) \
                else "No diagnostic provided"
            return f"{element_name.upper()}: {name} stream {self.my_id()} {d}"

        def current_stream_id():
            stream, _ = self.get_stream()
            return stream.stream_id

        if stream_event == StreamEvent.DROP_FRAME:
            return StreamState.DROP_FRAME
        if stream_event == StreamEvent.STOP:
            self.logger.debug(get_diagnostic())
            if not in_destroy_stream:
                self._post_message(ActorTopic.IN, "destroy_stream", [current_stream_id(), True])
            return StreamState.STOP
        if stream_event == StreamEvent.ERROR:
            self.logger.error(get_diagnostic())
            if not in_destroy_stream:
                stream, _ = self.get_stream()
                stream.state = StreamState.ERROR
                self.destroy_stream(current_stream_id(), use_thread_local=False)
            return StreamState.ERROR
        return StreamState.RUN

    def _release_frame(self, stream, frame_id, after=None):
        """A frame leaves the pipeline (completed, dropped or failed): its hop receive slots and
        FramePool slots go back (event-gated) and its admission credit is returned.  ``after``:
        the :class:`~aiko_services_amd.parallel.hop.Dropped` handle of a zero-copy send that
        may still read the frame's FramePool slot — its callbacks and admission credit are then
        handed to the hop plane, which runs them once that transfer completed (no wait)."""
        done = stream.frames.pop(frame_id, None)
        callbacks = []
        if done is not None:
            if done.hop_handles:
                _hop.plane().release(done.hop_handles)     # event-gated slot release
            callbacks.extend(done.on_complete)              # e.g. FramePool slots
        key = (stream.stream_id, frame_id)
        if after is not None:
            for callback in callbacks:
                after.then(callback)
            with self._admit_cv:
                # the credit stays counted until the zero-copy send completes (its FramePool slot
                # is still read): destroy_stream's bulk release must not hand it out early
                self._admit_deferred.add((str(key[0]), key[1]))
            after.then(lambda: self._admit_release(key))
            self._watch_hops()                              # the hop timer polls the transfer
            return
        for callback in callbacks:
            callback()
        self._admit_release(key)

    # ---- admission window (credits for generated frames) -----------------------------------------
    @property
    def admission_timeout(self) -> float:
        v, found = self.get_parameter("admission_timeout")
        try:
            return float(v) if found else 120.0
        except (TypeError, ValueError):
            return 120.0

    def limit_frames(self, owner: str, n: int) -> None:
        """An element caps the frames the pipeline may have in flight (e.g. SyntheticFrames:
        its FramePool slots, each held by a frame until it completes)."""
        with self._admit_cv:
            self._window_limits[owner] = max(1, int(n))
            self._admit_cv.notify_all()

    def frame_window(self) -> int:
        """Generated frames allowed in flight (0 = unlimited): the ``frame_window`` parameter,
        else the smallest element limit, else — with remote elements — twice the hop credits."""
        v, found = self.get_parameter("frame_window")
        if found:
            try:
                return max(0, int(v))
            except (TypeError, ValueError):
                pass
        if self._window_limits:
            return min(self._window_limits.values())
        if self.remote_pipelines:
            hop = _hop.plane()
            return 2 * (hop.depth if hop is not None else 4) * self.hop_batch * max(1, self._remote_member_count())
        return 0

    def _remote_member_count(self) -> int:
        return sum(len(r._members) for _, _, r in self.remote_pipelines.values() if r is not None)

    def admit_frame(self, stream_id, frame_id, timeout: float | None = None) -> bool:
        """Block the CALLING thread (a frame generator, a bench driver — never the actor) until
        the pipeline has fewer than :meth:`frame_window` admitted frames in flight; the frame
        ``(stream_id, frame_id)`` is then counted until it leaves the pipeline.  False on timeout."""
        key = (str(stream_id), frame_id)
        deadline = time.monotonic() + (self.admission_timeout if timeout is None else timeout)
        with self._admit_cv:
            while True:
                window = self.frame_window()
                if window <= 0 or len(self._admitted) < window:
                    self._admitted.add(key)
                    return True
                left = deadline - time.monotonic()
                if left <= 0:
                    return False
                self._admit_cv.wait(min(left, 0.5))

    def _admit_release(self, key):
        key = (str(key[0]), key[1])
        with self._admit_cv:
            self._admit_deferred.discard(key)
            if key in self._admitted:
                self._admitted.discard(key)
                self._admit_cv.notify_all()

    def _admit_release_stream(self, stream_id):
        """Every admission credit a destroyed stream still holds (frames admitted but rejected
        before they existed, or never released): the window is shared by the whole pipeline."""
        stream_id = str(stream_id)
        with self._admit_cv:
            stale = [k for k in self._admitted if k[0] == stream_id and k not in self._admit_deferred]
            if stale:
                self._admitted.difference_update(stale)
                self._admit_cv.notify_all()

    # ---- remote hops: credits, dispatch, failure ------------------------------------------------
    def _param_float(self, name, default):
        v, found = self.get_parameter(name)
        try:
            return float(v) if found else default
        except (TypeError, ValueError):
            return default

    def _has_credit(self, proxy) -> bool:
        if isinstance(proxy, LocalStage):
            return True
        rank = getattr(proxy, "hop_rank", None)
        hop = _hop.plane()
        if hop is not None and rank is not None:
            return hop.credit(rank) > 0
        window = int(self._param_float("remote_window", 0))
        if window <= 0:
            return True
        return sum(1 for f in self._inflight.values() if f["target"] is proxy) < window

    def _dispatch(self, element, target, node_name, stream_id, frame_id, inputs, held=False, ready=None):
        """Send frame ``(stream_id, frame_id)`` (paused at ``node_name``) to ``target``: metadata
        over MQTT, tensors over RCCL holding one of the target link's credits until the response
        (``held``: the frame's bytes are already staged — a re-dispatch).  ``ready``: the event
        of the stream that produced ``inputs`` when this runs from another stream (a queued
        frame dispatched from another frame's lane or the event loop).  A LocalStage target runs
        in-process and resumes the frame through ``process_frame_response``."""
        key = (stream_id, frame_id)
        if isinstance(target, LocalStage):
            hop = _hop.plane()
            values = hop.held_values(key) if held and hop is not None else inputs
            event_, out = target.run(stream_id, frame_id, values)
            if held and hop is not None:
                hop.drop(key)
            info = {"stream_id": stream_id, "frame_id": frame_id}
            if event_ == StreamEvent.ERROR:
                self._fail_frame(key, out.get("diagnostic", "local replica error") if isinstance(out, dict) else "")
                return
            self._post_message(ActorTopic.IN, "process_frame_response", [info, out],
                               target_function=self.process_frame_response)
            return
        stream_info = {"stream_id": stream_id, "frame_id": frame_id}
        hop = _hop.plane()
        rank = getattr(target, "hop_rank", None)
        out = inputs
        if hop is not None and rank is not None:
            # metadata over MQTT, tensors over RCCL to the remote's rank
            stream_info["hop_rank"] = hop.rank
            stream_info["reply_to"] = self.topic_in
            try:
                out = hop.resend(key, rank) if held else \
                    hop.encode(rank, inputs, key=key, ready=None if ready is None else [ready])
            except _hop.StageFailure as exc:
                self._replica_lost_rank(exc.peer)
                if not held:
                    self._queue_hop(element, node_name, stream_id, frame_id, inputs, ready=ready)
                return
        self._inflight[key] = {"element": element, "target": target, "node": node_name, "rank": rank,
                               "inputs": inputs if rank is None else None, "t": time.monotonic()}
        self._watch_hops()
        target.process_frame(stream_info, **out)

    def _queue_hop(self, element, node_name, stream_id, frame_id, inputs, held=False, ready=None):
        """Frame ``(stream_id, frame_id)`` waits for a credit of ``node_name``.  Its inputs are
        sent later from whichever stream drains the queue, so they are captured here, on the
        producing stream: tensors the producer may rewrite are copied into queue-owned
        storage and an event marks them written (``ready``: inputs already captured)."""
        limit = int(self._param_float("remote_pending", 256))
        if self._pending_total() >= limit:
            self.frames_dropped += 1
            self.logger.warning(f"remote {node_name}: {limit} frames already wait for a credit: dropping "
                                f"<{stream_id}:{frame_id}>")
            hop = _hop.plane()
            pending = hop.drop((stream_id, frame_id)) if held and hop is not None else None
            lease = self.stream_leases.get(str(stream_id))
            if lease is not None:
                self._release_frame(lease.stream, frame_id, after=pending)
            return
        hop = _hop.plane()
        if hop is not None and not held and ready is None:
            inputs, ready = hop.hold_inputs(inputs)
        self._pending_hops.setdefault(node_name, deque()).append({
                                   "element": element, "node": node_name, "stream_id": stream_id,
                                   "frame_id": frame_id, "inputs": inputs, "held": held,
                                   "ready": ready, "t": time.monotonic()})
        self._watch_hops()

    @property
    def hop_batch(self) -> int:
        """Frames per remote-hop message (pipeline parameter ``hop_batch``, default 1 = the
        reference's one message per frame).  Frames waiting for a credit leave in groups of up
        to this many: one control message, one transfer, ONE credit per group."""
        return max(1, int(self._param_float("hop_batch", 1)))

    def _pending_alive(self, p) -> bool:
        lease = self.stream_leases.get(str(p["stream_id"]))
        if lease is None or p["frame_id"] not in lease.stream.frames:
            if p["held"] and _hop.plane() is not None:
                _hop.plane().drop((p["stream_id"], p["frame_id"]))
            return False
        return True

    def _drain_pending(self):
        """Dispatch waiting frames while their remote element has a member with a credit
        (grouped up to :attr:`hop_batch` frames per message)."""
        if self._draining:
            return                       # re-entered (a replica lost mid-dispatch): the outer pass continues
        self._draining = True
        try:
            k = self.hop_batch
            for node_name, fifo in list(self._pending_hops.items()):
                while fifo:
                    p = fifo[0]
                    if not self._pending_alive(p):
                        fifo.popleft()
                        continue
                    element = self.pipeline_graph.get_node(node_name).element
                    target = element.pick(self._has_credit) if isinstance(element, RemoteReplicas) else None
                    if target is None:
                        break                # no member credit left: the FIFO waits
                    fifo.popleft()
                    group = [p]
                    if k > 1 and not p["held"] and getattr(target, "hop_rank", None) is not None:
                        while fifo and len(group) < k and not fifo[0]["held"]:
                            q = fifo.popleft()
                            if self._pending_alive(q):
                                group.append(q)
                    if len(group) == 1:
                        self._dispatch(element, target, node_name, p["stream_id"], p["frame_id"], p["inputs"],
                                       held=p["held"], ready=p.get("ready"))
                    else:
                        self._dispatch_group(element, target, node_name, group)
                if not fifo and self._pending_hops.get(node_name) is fifo:
                    del self._pending_hops[node_name]
        finally:
            self._draining = False

    def _pending_total(self) -> int:
        return sum(len(f) for f in self._pending_hops.values())

    def _dispatch_group(self, element, target, node_name, group):
        """Frames ``group`` (pending entries of one remote node) to ``target`` as ONE
        ``process_frames`` message whose tensors travel in ONE transfer holding ONE credit."""
        hop = _hop.plane()
        rank = target.hop_rank
        keys = [(g["stream_id"], g["frame_id"]) for g in group]
        try:
            outs = hop.encode_group(rank, [g["inputs"] for g in group], keys,
                                    ready=[g.get("ready") for g in group])
        except _hop.StageFailure as exc:
            self._replica_lost_rank(exc.peer)
            for g in group:
                self._queue_hop(element, node_name, g["stream_id"], g["frame_id"], g["inputs"],
                                ready=g.get("ready"))
            return
        now = time.monotonic()
        for key in keys:
            self._inflight[key] = {"element": element, "target": target, "node": node_name, "rank": rank,
                                   "inputs": None, "t": now}
        self.hop_groups += 1
        self._watch_hops()
        target.process_frames([{"stream_id": s, "frame_id": f, "hop_rank": hop.rank, "reply_to": self.topic_in}
                               for s, f in keys], outs)

    def _remote_done(self, key):
        f = self._inflight.pop(key, None)
        if f is None:
            return
        hop = _hop.plane()
        freed = True
        if hop is not None and f["rank"] is not None:
            freed = hop.ack(key)         # a group's credit returns with its last member
            if hop.dropped_inflight and hop.poll_dropped() == 0:
                freed = True             # dropped transfers finished: their credits are back
        if freed and self._pending_hops:
            self._drain_pending()

    def _fail_frame(self, key, diagnostic):
        """A frame that cannot complete (its replica died with no survivor to take it, or its
        hop timed out): StreamEvent.ERROR for its stream, as the reference does for a remote
        that errors (``/root/reference/src/aiko_services/main/pipeline.py:1229-1263``)."""
        self.hops_failed += 1
        hop = _hop.plane()
        pending = hop.drop(key) if hop is not None else None
        self._inflight.pop(key, None)
        lease = self.stream_leases.get(str(key[0]))
        if lease is None:
            # its stream is gone: only the admission credit is left
            if pending is not None:
                pending.then(lambda: self._admit_release(key))
            else:
                self._admit_release(key)
            return
        stream = lease.stream
        self._release_frame(stream, key[1], after=pending)
        self.logger.error(f"Frame <{key[0]}:{key[1]}>: {diagnostic}")
        if stream.state != StreamState.ERROR:
            stream.state = StreamState.ERROR
            if stream.queue_response is not None:
                stream.queue_response.put(({"stream_id": key[0], "frame_id": key[1], "state": StreamState.ERROR},
                                           {"diagnostic": diagnostic}))
            self.destroy_stream(str(key[0]), use_thread_local=False)

    def _rejoin_deadline(self, element_name, element_instance):
        """``rejoin_timeout`` after a stage lost its last member: still nobody back -> absent."""
        node = self.pipeline_graph.get_node(element_name)
        replicas = node.element if isinstance(node.element, RemoteReplicas) else None
        if replicas is None or not replicas.awaiting or replicas.members:
            return
        replicas.awaiting = False
        self.logger.warning(f"remote {element_name}: no replica rejoined: marking it absent")
        element_instance.set_remote_absent(True)
        node.element = element_instance
        self._update_lifecycle_state()

    def _replica_lost_rank(self, rank):
        """A hop peer failed (transport error): drop it from every remote element."""
        for service_name, (name, instance, replicas) in list(self.remote_pipelines.items()):
            if replicas is None:
                continue
            for topic, m in list(replicas._members.items()):
                if getattr(m[0], "hop_rank", None) == rank:
                    self._replica_lost(service_name, topic)

    def _replica_lost(self, service_name, topic_path):
        """Member ``topic_path`` of a remote element is gone (registrar remove / last will, or
        a transport error): retire its RCCL links (no wait on its pending transfers can reach a
        live stream), then re-dispatch every frame it held to a survivor — its staged bytes are
        re-sent, not recomputed — or queue it for a credit; the element drops to absent (and the
        pipeline's lifecycle to waiting) when no member is left.  Reference: the remote swap to
        the absent proxy, ``/root/reference/src/aiko_services/main/pipeline.py:975-1006``."""
        element_name, element_instance, replicas = self.remote_pipelines[service_name]
        member = replicas._members.get(topic_path) if replicas is not None else None
        if member is None:
            return
        proxy = member[0]
        replicas.remove(topic_path)
        # degraded but serving: the survivors are the stage now (``expected`` only gates start-up)
        replicas.expected = min(replicas.expected, len(replicas._members))
        rank = getattr(proxy, "hop_rank", None)
        hop = _hop.plane()
        if hop is not None and rank is not None:
            hop.mark_dead(rank)
        node = self.pipeline_graph.get_node(element_name)
        if replicas.members or (rank is not None and _supervised()):
            # (supervised: the dead rank is restarted — its frames wait for it, up to hop_timeout)
            replicas.awaiting = not replicas.members
            node.element = replicas
            if replicas.awaiting:
                # bounded: if no member is back by rejoin_timeout (the supervisor gave up, or the
                # restart failed) the element is absent again, so frames fail at once instead of
                # each waiting out hop_timeout
                limit = self._param_float("rejoin_timeout", 120.0)
                self._post_message(ActorTopic.IN, "rejoin_deadline", [element_name, element_instance],
                                   delay=limit, target_function=self._rejoin_deadline)
        else:
            element_instance.set_remote_absent(True)
            node.element = element_instance
        self._update_lifecycle_state()
        lost = [(k, f) for k, f in self._inflight.items() if f["target"] is proxy]
        for key, f in lost:
            self._inflight.pop(key, None)
            held = f["rank"] is not None
            inputs = f["inputs"]
            if held and hop is not None and hop.grouped(key):
                # a group member: re-sent on its own from views of the group's staging buffer
                inputs = hop.held_values(key)
                hop.ack(key)
                held = False
            self.hops_redispatched += 1
            self._queue_hop(f["element"], f["node"], key[0], key[1], inputs, held=held)
        if lost:
            self.logger.warning(f"remote {element_name}: member {topic_path} lost with {len(lost)} frames "
                                f"in flight: re-dispatching")
        self._drain_pending()

    def _watch_hops(self):
        if not self._hop_watch:
            self._hop_watch = True
            event.add_timer_handler(self._hop_timer, 0.5)

    def _hop_timer(self):
        """Hop timeout (``hop_timeout`` s, default 60): a frame whose remote response or credit
        never comes ends with StreamEvent.ERROR instead of holding its stream forever."""
        timeout = self._param_float("hop_timeout", 60.0)
        now = time.monotonic()
        hop = _hop.plane()
        if hop is not None and hop.dropped_inflight:
            before = hop.dropped_inflight
            if hop.poll_dropped() < before and self._pending_hops:
                self._drain_pending()    # credits of finished dropped transfers came back
        for key, f in list(self._inflight.items()):
            if now - f["t"] > timeout:
                escalate = False
                if hop is not None and f["rank"] is not None:
                    # alive but unresponsive: no new frames for it, bar one probe frame every
                    # AIKO_HOP_PROBE_S; unanswered probes retire it (supervised restart)
                    escalate = hop.suspend(f["rank"])
                self._fail_frame(key, f"remote hop to {f['node']} timed out after {timeout:g}s")
                if escalate:
                    self.logger.warning(f"remote {f['node']}: rank {f['rank']} answered no probe: retiring it")
                    self._replica_lost_rank(f["rank"])
        if self._pending_hops:
            self._drain_pending()
            for fifo in list(self._pending_hops.values()):
                for p in list(fifo):
                    if now - p["t"] > timeout:
                        fifo.remove(p)
                        self._fail_frame((p["stream_id"], p["frame_id"]),
                                         f"no replica of {p['node']} had a credit for {timeout:g}s")
            for node_name in [n for n, f in self._pending_hops.items() if not f]:
                del self._pending_hops[node_name]
        if not self._inflight and not self._pending_hops and not (hop is not None and hop.dropped_inflight):
            self._hop_watch = False
            event.remove_timer_handler(self._hop_timer)

    # ---- parameters ------------------------------------------------------------------------------
    def set_parameter(self, stream_id, name, value):
        if stream_id is None:
            names = str(name).split(".")
            if len(names) == 1:
                self.ec_producer.update(names[0], value)
            else:
                try:
                    element = self.pipeline_graph.get_node(names[0]).element
                    element.ec_producer.update(names[1], value)
                except (KeyError, AttributeError):
                    pass
        else:
            lease = self.stream_leases.get(str(stream_id))
            if lease is not None:
                lease.stream.parameters[name] = value

    def set_parameters(self, stream_id, parameters):
        for p in parameters or []:
            self.set_parameter(stream_id, p[0], p[1])

    def get_element(self, name):
        return self.pipeline_graph.get_node(name).element

    def set_remote_replicas(self, element_name, expected: int, local_definition=None, local_weight=0.0):
        """Remote element ``element_name`` is a replicated stage: wait for ``expected`` members
        (remote services + the local copy) before it is ready; with ``local_definition`` (a
        PipelineDefinition) a copy of the stage runs in this process taking ``local_weight``
        of the frames (``parallel/placement.py``)."""
        for service_name, (name, instance, replicas) in list(self.remote_pipelines.items()):
            if name != element_name:
                continue
            if replicas is None:
                replicas = RemoteReplicas(instance.definition)
            replicas.expected = int(expected)
            if local_definition is not None and local_weight > 0:
                child = PipelineImpl.create_pipeline("<local_stage>", local_definition,
                                                     f"{local_definition.name}_local", None, None, [], 0,
                                                     None, GRACE_TIME)
                child.response_swag = getattr(self, "response_swag", False)
                replicas.add("local", LocalStage(child), weight=local_weight)
            self.remote_pipelines[service_name] = (name, instance, replicas)
            if replicas.members:
                self.pipeline_graph.get_node(name).element = replicas
            self._update_lifecycle_state()
            return replicas
        raise KeyError(f"no remote element {element_name}")


# ---- remote element placeholder --------------------------------------------------------------

def _supervised() -> bool:
    """Whether dead ranks are restarted (``AIKO_SUPERVISE``, see ``parallel/launch.py``)."""
    try:
        return int(os.environ.get("AIKO_SUPERVISE", "0") or 0) > 0
    except ValueError:
        return False


class RemoteReplicas:
    """The discovered instances of one remote PipelineElement.

    The reference binds a remote element to the single service its filter finds
    (``/root/reference/src/aiko_services/main/pipeline.py:686-714``).  Here every matching
    service is a member: streams are created / destroyed on all of them and each frame goes to
    one, chosen by smooth weighted round-robin (service tag ``weight=w``, default 1) — a
    replicated pipeline stage (PP x DP).  With one member this is exactly the reference hop.
    """

    def __init__(self, definition, expected: int = 1):
        self.definition = definition
        self.expected = expected        # members needed before the element counts as ready
        self._members: "OrderedDict[str, list]" = OrderedDict()    # topic_path -> [proxy, weight, credit]
        self.awaiting = False           # every member lost, a supervised restart will bring one back


    @property
    def members(self):
        return self._members if len(self._members) >= self.expected else {}

    def add(self, topic_path, proxy, weight: float = 1.0):
        self._members[topic_path] = [proxy, max(1e-6, float(weight)), 0.0]
        self.awaiting = False

    def remove(self, topic_path) -> bool:
        return self._members.pop(topic_path, None) is not None

    def pick(self, available=None):
        """Smooth weighted round-robin over the members ``available(proxy)`` accepts (those
        with a credit left); None when there is none."""
        total = 0.0
        best = None
        for m in self._members.values():
            if available is not None and not available(m[0]):
                continue
            m[2] += m[1]
            total += m[1]
            if best is None or m[2] > best[2]:
                best = m
        if best is None:
            return None
        best[2] -= total
        return best[0]

    @property
    def proxies(self):
        return [m[0] for m in self._members.values()]

    def create_stream(self, *args, **kwargs):
        for p in self.proxies:
            p.create_stream(*args, **kwargs)

    def destroy_stream(self, *args, **kwargs):
        for p in self.proxies:
            p.destroy_stream(*args, **kwargs)

    def __repr__(self):
        return f"RemoteReplicas({list(self._members)})"


class LocalStage:
    """Member of a :class:`RemoteReplicas` that runs the replicated stage inside this process:
    a child Pipeline built from the stage's definition, called synchronously (its graph must be
    fully local).  Lets rank 0 take a share of the frames of the stage it feeds."""

    def __init__(self, pipeline):
        import queue as _queue
        self.pipeline = pipeline
        self.responses = _queue.Queue()
        self.hop_rank = None

    def create_stream(self, stream_id, graph_path=None, parameters=None, grace_time=GRACE_TIME,
                      queue_response=None, topic_response=None):
        self.pipeline.create_stream(stream_id, None, parameters, grace_time, queue_response=self.responses)

    def destroy_stream(self, stream_id, graceful=False):
        self.pipeline.destroy_stream(stream_id, graceful)

    def run(self, stream_id, frame_id, inputs):
        self.pipeline.process_frame({"stream_id": stream_id, "frame_id": frame_id}, dict(inputs))
        try:
            info, out = self.responses.get_nowait()
        except Exception:
            return StreamEvent.ERROR, {"diagnostic": "local stage replica produced no response"}
        state = int(info.get("state", 0))
        event_ = {StreamState.DROP_FRAME: StreamEvent.DROP_FRAME, StreamState.ERROR: StreamEvent.ERROR,
                  StreamState.STOP: StreamEvent.STOP}.get(state, StreamEvent.OKAY)
        return event_, dict(out)


class PipelineRemote(PipelineElement):

    def __init__(self, context):
        context.get_implementation("PipelineElement").__init__(self, context)
        self.set_remote_absent(True)

    def create_stream(self, stream_id, graph_path=None, parameters=None, grace_time=GRACE_TIME,
                      queue_response=None, topic_response=None):
        if self.absent:
            self.log_error("create_stream")
        return not self.absent

    def destroy_stream(self, stream_id, graceful=False):
        if self.absent:
            self.log_error("destroy_stream")
        return not self.absent

    @classmethod
    def is_local(cls):
        return False

    def log_error(self, function_name):
        self.logger.error(f"PipelineElement.{function_name}(): {self.definition.name}: invoked when "
                          "remote Pipeline hasn't been discovered")

    def process_frame(self, stream, **kwargs):
        if self.absent:
            self.log_error("process_frame")
        return not self.absent

    def process_frame_response(self, stream, frame_data):
        pass

    def process_frames(self, stream_dicts, frame_datas):
        """A hop group (see ``PipelineImpl.process_frames``)."""
        if self.absent:
            self.log_error("process_frames")
        return not self.absent

    def set_remote_absent(self, absent):
        self.absent = absent
        self.share["lifecycle"] = "absent" if absent else "ready"
