"""L0 utilities: S-expression codec, graph, configuration, logging, importer, misc helpers."""
from .configuration import *  # noqa: F401,F403
from .graph import Graph, Node  # noqa: F401
from .logger import *  # noqa: F401,F403
from .misc import *  # noqa: F401,F403
from .sexpr import generate, parse, parse_float, parse_int, parse_number  # noqa: F401

# reference module name alias: aiko_services.main.utilities.parser
from . import sexpr as parser  # noqa: F401,E402
