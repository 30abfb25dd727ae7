"""L2/L3 runtime: event engine, process singleton, composition, services, actors, leases."""
from . import event  # noqa: F401
from .connection import Connection, ConnectionState  # noqa: F401
from .context import *  # noqa: F401,F403
from .fsm import StateMachine  # noqa: F401
from .process import ProcessData, ProcessImplementation, aiko, process_create  # noqa: F401
from .service import *  # noqa: F401,F403
from .lease import Lease  # noqa: F401
from .actor import *  # noqa: F401,F403
from .proxy import ProxyAllMethods, is_callable, proxy_timing, proxy_trace  # noqa: F401
