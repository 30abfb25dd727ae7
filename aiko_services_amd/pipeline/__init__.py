"""L6 dataflow engine: definitions, streams, Pipeline/PipelineElement, CLI."""
from .definition import *  # noqa: F401,F403
from .stream import *  # noqa: F401,F403
from .engine import *  # noqa: F401,F403
