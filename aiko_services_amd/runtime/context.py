"""Context dataclasses, Interface defaults and FrankensteinClass composition.

Reference: ``main/context.py:56-190`` (Context, Interface, ContextService,
ContextPipelineElement, ContextPipeline, ``*_args`` builders) and ``main/component.py:50-219``
(``compose_class`` / ``compose_instance``).  Semantics preserved so user classes written
against the reference compose identically:

* ``Interface.default(name, impl)`` registers a process-wide default implementation (the
  reference's ``Interface.context`` is one shared class attribute);
* ``compose_class(seed, overrides)`` keeps only implementations of interfaces in the seed's
  MRO, refuses unimplemented interfaces, loads dotted-path implementations, and adds each
  implementation's methods to a subclass of the seed only where the seed's attribute is
  missing or abstract, then recomputes ``__abstractmethods__``.
"""
from __future__ import annotations

import abc
from abc import ABC
from dataclasses import dataclass, field
from inspect import getmembers, isclass, isfunction
from typing import Dict, List

__all__ = [
    "Context", "Interface", "ServiceProtocolInterface", "ContextService",
    "ContextPipelineElement", "ContextPipeline", "service_args", "actor_args",
    "pipeline_element_args", "pipeline_args", "compose_class", "compose_instance",
    "DEFAULT_PROTOCOL", "DEFAULT_TRANSPORT",
]

DEFAULT_PROTOCOL = "*"
DEFAULT_TRANSPORT = "mqtt"
DEFAULT_DEFINITION = ""
DEFAULT_DEFINITION_PATHNAME = ""


@dataclass
class Context:
    name: str = "<interface>"
    implementations: Dict[str, object] = field(default_factory=dict)

    def get_implementation(self, implementation_name):
        return self.implementations[implementation_name]

    def get_implementations(self):
        return self.implementations

    def get_name(self) -> str:
        return self.name

    def set_implementation(self, implementation_name, implementation):
        self.implementations[implementation_name] = implementation

    def set_implementations(self, implementations):
        self.implementations = implementations


class Interface(ABC):
    context = Context()   # shared by every Interface subclass (process-wide defaults)

    @classmethod
    def default(cls, implementation_name, implementation):
        cls.context.set_implementation(implementation_name, implementation)

    @classmethod
    def get_implementations(cls):
        return cls.context.get_implementations()


class ServiceProtocolInterface(Interface):
    """Interface marker: an Aiko Service implementing a protocol."""


@dataclass
class ContextService(Context):
    parameters: Dict[str, str] = field(default_factory=dict)
    protocol: str = DEFAULT_PROTOCOL
    tags: List[str] = field(default_factory=list)
    transport: str = DEFAULT_TRANSPORT

    def __post_init__(self):
        if self.name is None or not isinstance(self.name, str):
            raise ValueError(f"Service name must be a string: {self.name}")
        if not self.name:
            raise ValueError("Service name must not be an empty string")
        if self.implementations is None:
            self.implementations = {}
        if self.parameters is None:
            self.parameters = {}
        if self.protocol is None:
            self.protocol = DEFAULT_PROTOCOL
        if self.tags is None:
            self.tags = []
        else:
            self.tags = list(self.tags)
        if self.transport is None:
            self.transport = DEFAULT_TRANSPORT

    def get_parameters(self):
        return self.parameters

    def get_protocol(self):
        return self.protocol

    def get_tags(self):
        return self.tags

    def get_transport(self):
        return self.transport

    def set_protocol(self, protocol):
        self.protocol = protocol


@dataclass
class ContextPipelineElement(ContextService):
    definition: object = DEFAULT_DEFINITION
    pipeline: object = None

    def __post_init__(self):
        self.name = self.name.lower() if isinstance(self.name, str) else self.name
        super().__post_init__()
        if self.definition is None:
            self.definition = DEFAULT_DEFINITION

    def get_definition(self):
        return self.definition

    def get_pipeline(self):
        return self.pipeline


@dataclass
class ContextPipeline(ContextPipelineElement):
    definition_pathname: str = DEFAULT_DEFINITION_PATHNAME
    graph_path: str = None

    def __post_init__(self):
        super().__post_init__()
        if self.definition_pathname is None:
            self.definition_pathname = DEFAULT_DEFINITION_PATHNAME

    def get_definition_pathname(self):
        return self.definition_pathname

    def get_graph_path(self):
        return self.graph_path


def service_args(name, implementations=None, parameters=None, protocol=None, tags=None,
                 transport=None):
    return {"context": ContextService(name, implementations, parameters, protocol, tags, transport)}


def actor_args(name, implementations=None, parameters=None, protocol=None, tags=None,
               transport=None):
    return service_args(name, implementations, parameters, protocol, tags, transport)


def pipeline_element_args(name, implementations=None, parameters=None, protocol=None, tags=None,
                          transport=None, definition=None, pipeline=None):
    return {"context": ContextPipelineElement(name, implementations, parameters, protocol, tags,
                                              transport, definition, pipeline)}


def pipeline_args(name, implementations=None, parameters=None, protocol=None, tags=None,
                  transport=None, definition=None, pipeline=None, definition_pathname=None,
                  graph_path=None):
    return {"context": ContextPipeline(name, implementations, parameters, protocol, tags,
                                       transport, definition, pipeline, definition_pathname,
                                       graph_path)}


# ---- composition ----------------------------------------------------------------------------

def _is_abstract(attr) -> bool:
    return bool(getattr(attr, "__isabstractmethod__", False))


def _is_interface(cls) -> bool:
    """A class whose every function is abstract (vacuously true for marker classes)."""
    return all(_is_abstract(m) for _, m in getmembers(cls, isfunction))


_BASE_MARKERS = (ABC, Interface, ServiceProtocolInterface, object)


def _keep_specified_implementations(seed, implementations):
    kept = {}
    for ancestor in seed.__mro__:
        name = ancestor.__name__
        if name in implementations and _is_interface(ancestor):
            kept[name] = implementations[name]
    return kept


def _check_interfaces_implemented(seed, implementations):
    missing = []
    for ancestor in seed.__mro__:
        if ancestor in _BASE_MARKERS:
            continue
        if _is_interface(ancestor) and ancestor.__name__ not in implementations:
            missing.append(ancestor.__name__)
    return missing


def _load_implementations(implementations):
    from ..utils.misc import load_module
    loaded = {}
    for alias, impl in implementations.items():
        if isclass(impl):
            loaded[alias] = impl
            continue
        module_name, _, class_name = str(impl).rpartition(".")
        if not module_name:
            raise ValueError(f"For {alias} interface, the implementation module name must be provided: {impl}")
        loaded[alias] = getattr(load_module(module_name), class_name)
    return loaded


def _add_methods(base, implementations):
    for impl in implementations.values():
        for name, fn in getmembers(impl, isfunction):
            if name.startswith("__"):
                continue
            current = getattr(base, name, None)
            if current is None or _is_abstract(current):
                setattr(base, name, fn)


def compose_class(impl_seed_class, impl_overrides=None):
    all_impls = {**impl_seed_class.get_implementations(), **(impl_overrides or {})}
    impls = _keep_specified_implementations(impl_seed_class, all_impls)
    missing = _check_interfaces_implemented(impl_seed_class, impls)
    if missing:
        raise ValueError(f"Unimplemented interfaces: {', '.join(missing)}")
    loaded = _load_implementations(impls)

    class FrankensteinClass(impl_seed_class):
        pass

    _add_methods(FrankensteinClass, loaded)
    FrankensteinClass.__init__ = impl_seed_class.__init__
    abc.update_abstractmethods(FrankensteinClass)
    FrankensteinClass.__name__ = impl_seed_class.__name__
    FrankensteinClass.__qualname__ = impl_seed_class.__qualname__
    return FrankensteinClass, loaded


def compose_instance(impl_seed_class, init_args, impl_overrides=None):
    cls, implementations = compose_class(impl_seed_class, impl_overrides)
    init_args["context"].set_implementations(implementations)
    return cls(**init_args)
