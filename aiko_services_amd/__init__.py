"""aiko_services_amd — an MI355X-native actor / dataflow-pipeline framework.

Public API parity with the reference package facade (``aiko_services/main/__init__.py``):
``import aiko_services_amd as aiko`` (or the compatibility alias ``import aiko_services as
aiko``) exposes Context/Interface composition, the event engine, ``aiko`` / ``aiko.process``,
Services, Actors, leases, EC share, the registrar, lifecycle management, streams and the
Pipeline / PipelineElement engine.  The GPU data plane lives in :mod:`aiko_services_amd.gpu`,
:mod:`aiko_services_amd.ops` (HIP kernels), :mod:`aiko_services_amd.models` and
:mod:`aiko_services_amd.parallel` (RCCL over xGMI); none of it is imported here, so control-
plane-only processes never load torch.
"""
__version__ = "0.1.0"

from .runtime.context import (Context, ContextPipeline, ContextPipelineElement, ContextService,  # noqa: F401
                              Interface, ServiceProtocolInterface, actor_args, compose_class,
                              compose_instance, pipeline_args, pipeline_element_args, service_args)
from .runtime.connection import Connection, ConnectionState  # noqa: F401
from .runtime.event import (add_flatout_handler, add_mailbox_handler, add_queue_handler,  # noqa: F401
                            add_timer_handler, loop, mailbox_put, queue_put, remove_flatout_handler,
                            remove_mailbox_handler, remove_queue_handler, remove_timer_handler,
                            terminate)
from .runtime import event  # noqa: F401
from .runtime.process import aiko, process_create  # noqa: F401
from .runtime.lease import Lease  # noqa: F401
from .runtime.service import (Service, ServiceFields, ServiceFilter, ServiceImpl, ServiceProtocol,  # noqa: F401
                              Services, ServiceTags, ServiceTopicPath)
from .runtime.fsm import StateMachine  # noqa: F401
from .runtime.proxy import ProxyAllMethods, is_callable, proxy_trace  # noqa: F401
from .control.share import (PROTOCOL_EC_CONSUMER, PROTOCOL_EC_PRODUCER, ECConsumer, ECProducer,  # noqa: F401
                            services_cache_create_singleton, services_cache_delete)
from .runtime.actor import Actor, ActorImpl, ActorTest, ActorTestImpl, ActorTopic  # noqa: F401
from .control.process_manager import ProcessManager  # noqa: F401
from .control.lifecycle import LifeCycleClient, LifeCycleManager  # noqa: F401
from .control.transport import (ActorDiscovery, TransportMQTT, TransportMQTTImpl,  # noqa: F401
                                get_actor_mqtt)
from .pipeline.stream import (DEFAULT_STREAM_ID, FIRST_FRAME_ID, Frame, Stream, StreamEvent,  # noqa: F401
                              StreamEventName, StreamState, StreamStateName)
from .pipeline.engine import (PROTOCOL_PIPELINE, Pipeline, PipelineElement,  # noqa: F401
                              PipelineElementImpl, PipelineImpl, PipelineRemote)
from .control.registrar import Registrar, RegistrarImpl, REGISTRAR_PROTOCOL  # noqa: F401
from .utils import (Graph, Node, generate, get_hostname, get_logger, get_namespace, get_pid,  # noqa: F401
                    get_username, parse, parse_float, parse_int, parse_number)

aiko.process = process_create()
process = aiko.process
