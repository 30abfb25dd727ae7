"""Compatibility alias: ``import aiko_services as aiko`` resolves to :mod:`aiko_services_amd`.

Users switching from the reference keep their imports, and PipelineDefinition JSON files that
name modules such as ``aiko_services.elements.media.text_io`` or
``aiko_services.examples.pipeline.elements`` load the MI355X-native implementations.  This is
a module-path alias only (a meta-path finder mapping names), not a translation layer.
"""
import importlib
import importlib.abc
import importlib.util
import sys

_PREFIX = "aiko_services"
_TARGET = "aiko_services_amd"

# reference module path (after "aiko_services.") -> module inside aiko_services_amd
_MAP = {
    "main": "",
    "main.utilities": "utils",
    "main.utilities.parser": "utils.sexpr",
    "main.utilities.graph": "utils.graph",
    "main.utilities.configuration": "utils.configuration",
    "main.utilities.logger": "utils.logger",
    "main.utilities.importer": "utils.misc",
    "main.utilities.lock": "utils.misc",
    "main.utilities.lru_cache": "utils.misc",
    "main.utilities.context": "utils.misc",
    "main.utilities.network": "utils.misc",
    "main.utilities.utc_iso8601": "utils.misc",
    "main.context": "runtime.context",
    "main.component": "runtime.context",
    "main.connection": "runtime.connection",
    "main.event": "runtime.event",
    "main.process": "runtime.process",
    "main.service": "runtime.service",
    "main.actor": "runtime.actor",
    "main.lease": "runtime.lease",
    "main.proxy": "runtime.proxy",
    "main.state": "runtime.fsm",
    "main.share": "control.share",
    "main.registrar": "control.registrar",
    "main.lifecycle": "control.lifecycle",
    "main.process_manager": "control.process_manager",
    "main.transport": "control.transport",
    "main.transport.transport_mqtt": "control.transport",
    "main.message": "message",
    "main.message.mqtt": "message.message",
    "main.message.castaway": "message.message",
    "main.message.message": "message.message",
    "main.stream": "pipeline.stream",
    "main.pipeline": "pipeline.engine",
    "main.dashboard": "tools.dashboard",
    "main.recorder": "tools.recorder",
    "main.storage": "tools.storage",
    "main.cli": "tools.cli",
}


def _target_name(fullname):
    rest = fullname[len(_PREFIX) + 1:]
    mapped = _MAP.get(rest, rest)
    return _TARGET if mapped == "" else f"{_TARGET}.{mapped}"


class _AliasLoader(importlib.abc.Loader):
    def __init__(self, target):
        self.target = target

    def create_module(self, spec):
        return importlib.import_module(self.target)

    def exec_module(self, module):
        pass


class _AliasFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, fullname, path=None, target=None):
        if not fullname.startswith(_PREFIX + "."):
            return None
        tname = _target_name(fullname)
        if importlib.util.find_spec(tname) is None:
            return None
        spec = importlib.util.spec_from_loader(fullname, _AliasLoader(tname))
        target_spec = importlib.util.find_spec(tname)
        if target_spec is not None and target_spec.submodule_search_locations is not None:
            spec.submodule_search_locations = list(target_spec.submodule_search_locations)
        return spec


if not any(isinstance(f, _AliasFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _AliasFinder())

from aiko_services_amd import *  # noqa: F401,F403,E402
from aiko_services_amd import aiko, process  # noqa: F401,E402
