"""Local method-intercepting proxies (reference ``main/proxy.py``; no ``wrapt`` dependency).

``ProxyAllMethods(name, obj, proxy_function)`` forwards attribute access to ``obj`` but routes
every public bound method through ``proxy_function(name, obj, fn, fn_name, *args, **kw)`` —
e.g. ``proxy_trace`` (enter/exit tracing) or ``ActorImpl.proxy_post_message`` (turn local calls
into mailbox posts so they run on the actor's event loop).
"""
from __future__ import annotations

import time
from inspect import getmembers, isfunction, ismethod

__all__ = ["is_callable", "ProxyAllMethods", "proxy_trace", "proxy_timing"]


def is_callable(attribute):
    return isfunction(attribute) or ismethod(attribute)


class ProxyAllMethods:
    def __init__(self, proxy_name, actual_object, proxy_function, attribute_filter=ismethod,
                 ignore_prefix="_"):
        object.__setattr__(self, "_proxy_target", actual_object)
        object.__setattr__(self, "_proxy_name", proxy_name)
        wrapped = {}
        for name, fn in getmembers(actual_object, attribute_filter):
            if ignore_prefix is None or not name.startswith(ignore_prefix):
                def closure(*args, _fn=fn, _name=name, **kwargs):
                    return proxy_function(proxy_name, actual_object, _fn, _name, *args, **kwargs)
                wrapped[name] = closure
        object.__setattr__(self, "_proxy_methods", wrapped)

    def __getattr__(self, name):
        methods = object.__getattribute__(self, "_proxy_methods")
        if name in methods:
            return methods[name]
        return getattr(object.__getattribute__(self, "_proxy_target"), name)

    def __setattr__(self, name, value):
        setattr(object.__getattribute__(self, "_proxy_target"), name, value)

    @property
    def __wrapped__(self):
        return object.__getattribute__(self, "_proxy_target")

    def __repr__(self):
        return f"[{type(self).__module__}.{type(self).__name__} object at {hex(id(self))}]"


def proxy_trace(proxy_name, actual_object, actual_function, actual_function_name, *args, **kwargs):
    print(f"### Enter: {proxy_name}.{actual_function_name}{args} {kwargs} ###")
    try:
        return actual_function(*args, **kwargs)
    finally:
        print(f"### Exit:  {proxy_name}.{actual_function_name} ###")


def proxy_timing(proxy_name, actual_object, actual_function, actual_function_name, *args, **kwargs):
    """Accumulate per-method wall time in ``actual_object._proxy_timing`` (profiling aid)."""
    t0 = time.perf_counter()
    try:
        return actual_function(*args, **kwargs)
    finally:
        stats = actual_object.__dict__.setdefault("_proxy_timing", {})
        n, total = stats.get(actual_function_name, (0, 0.0))
        stats[actual_function_name] = (n + 1, total + time.perf_counter() - t0)
