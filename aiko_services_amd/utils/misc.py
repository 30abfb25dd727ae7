"""Small utilities: importer, named lock, LRU cache, context manager, network ports, UTC times.

Behaviour follows the reference ``utilities/{importer,lock,lru_cache,context,network,
utc_iso8601}.py``.
"""
from __future__ import annotations

import datetime as _dt
import importlib
import importlib.util
import os
import sys
import threading
import time
from collections import OrderedDict
from pathlib import Path

__all__ = [
    "load_module", "load_modules", "Lock", "LRUCache", "ContextManager", "get_context",
    "get_network_ports_listen", "datetime_now_utc_iso", "epoch_to_utc_iso",
    "utc_iso_to_datetime", "utc_iso_to_epoch",
]

# ---- importer (reference utilities/importer.py:19-47) -------------------------------------

_modules: dict = {}

# Module paths inside reference PipelineDefinitions ("aiko_services.elements.media...") resolve
# to this package through the aiko_services alias package (see aiko_services/__init__.py).


def load_module(module_descriptor: str):
    """Load ``pkg.module`` or ``path/to/file.py`` (cached)."""
    if module_descriptor in _modules:
        return _modules[module_descriptor]
    if os.environ.get("AIKO_IMPORTER_USE_CURRENT_DIRECTORY") and os.getcwd() not in sys.path:
        sys.path.append(os.getcwd())
    if module_descriptor.endswith(".py"):
        path = Path(module_descriptor)
        if not path.exists():
            raise FileNotFoundError(module_descriptor)
        name = path.stem
        spec = importlib.util.spec_from_file_location(name, str(path))
        module = importlib.util.module_from_spec(spec)
        sys.modules.setdefault(name, module)
        spec.loader.exec_module(module)
    else:
        if module_descriptor.startswith("aiko_services.") or module_descriptor == "aiko_services":
            import aiko_services  # noqa: F401  (installs the alias finder)
        module = importlib.import_module(module_descriptor)
    _modules[module_descriptor] = module
    return module


def load_modules(module_descriptors):
    return [load_module(m) for m in module_descriptors]


# ---- named lock that reports contention (reference utilities/lock.py) -----------------------

class Lock:
    def __init__(self, name, logger=None):
        self._name = name
        self._logger = logger
        self._lock = threading.RLock()
        self._in_use = None
        self.contention_count = 0

    def acquire(self, location=None):
        if not self._lock.acquire(blocking=False):
            self.contention_count += 1
            if self._logger:
                self._logger.debug(f"Lock {self._name}: {location} waiting, in use by {self._in_use}")
            self._lock.acquire()
        self._in_use = location

    def release(self):
        self._in_use = None
        self._lock.release()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


# ---- LRU cache (reference utilities/lru_cache.py) --------------------------------------------

class LRUCache:
    def __init__(self, size=128):
        self.size = size
        self.cache: OrderedDict = OrderedDict()

    def get(self, key, default=None):
        if key not in self.cache:
            return default
        self.cache.move_to_end(key)
        return self.cache[key]

    def put(self, key, value):
        self.cache[key] = value
        self.cache.move_to_end(key)
        while len(self.cache) > self.size:
            self.cache.popitem(last=False)

    def get_list(self):
        return list(self.cache.values())

    def __contains__(self, key):
        return key in self.cache

    def __len__(self):
        return len(self.cache)


# ---- global "current context" (reference utilities/context.py) ------------------------------

class ContextManager:
    _instance = None

    def __init__(self, aiko=None, message=None):
        self.aiko = aiko
        self.message = message
        ContextManager._instance = self

    def get_aiko(self):
        return self.aiko

    def get_message(self):
        return self.message


def get_context():
    return ContextManager._instance


# ---- network ports (reference utilities/network.py) -----------------------------------------

def get_network_ports_listen(kind="inet"):
    try:
        import psutil
    except ImportError:  # pragma: no cover
        return []
    ports = []
    for conn in psutil.net_connections(kind=kind):
        if conn.status == psutil.CONN_LISTEN or conn.type == 2:  # SOCK_DGRAM
            if conn.laddr:
                ports.append((conn.laddr.ip, conn.laddr.port, conn.pid))
    return sorted(set(ports))


# ---- UTC ISO-8601 helpers (reference utilities/utc_iso8601.py) ------------------------------

def datetime_now_utc_iso() -> str:
    return _dt.datetime.now(_dt.timezone.utc).isoformat()


def epoch_to_utc_iso(epoch: float) -> str:
    return _dt.datetime.fromtimestamp(epoch, _dt.timezone.utc).isoformat()


def utc_iso_to_datetime(iso: str) -> _dt.datetime:
    return _dt.datetime.fromisoformat(iso)


def utc_iso_to_epoch(iso: str) -> float:
    return utc_iso_to_datetime(iso).timestamp()


def monotonic() -> float:
    return time.monotonic()
