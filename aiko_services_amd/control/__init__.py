"""L4/L5 control plane: EC share, registrar, discovery, remote proxies, lifecycle, supervision."""
from .share import *  # noqa: F401,F403
from .transport import *  # noqa: F401,F403
from .registrar import Registrar, RegistrarImpl, REGISTRAR_PROTOCOL  # noqa: F401
