"""Remote actor proxies and actor discovery over the MQTT control plane.

Reference ``main/transport/transport_mqtt.py:49-141``.  ``get_actor_mqtt(topic_in, Interface)``
returns an object whose public methods (taken from the interface class) publish
``(method arg ...)`` S-expressions to ``topic_in``.  ``ActorDiscovery(service)`` wraps the
registrar ServicesCache with filter-based change callbacks ``handler(command, details)``.

Keyword arguments are encoded like the reference (``(method arg0 (k: v ...))``) but positional
arguments after the first are no longer dropped.
"""
from __future__ import annotations

from abc import abstractmethod  # noqa: F401
from inspect import getmembers, isfunction

from ..runtime.actor import Actor
from ..runtime.context import Interface
from ..runtime.process import aiko
from ..message.tensor_payload import encode_message
from ..utils.sexpr import generate
from .share import services_cache_create_singleton

__all__ = ["TransportMQTT", "TransportMQTTImpl", "ActorDiscovery", "ServiceDiscovery",
           "get_actor_mqtt", "get_public_methods", "make_proxy_mqtt", "ServiceRemoteProxy"]


class TransportMQTT(Actor):
    Interface.default("TransportMQTT", "aiko_services_amd.control.transport.TransportMQTTImpl")


class TransportMQTTImpl(TransportMQTT):
    def __init__(self, context):
        context.get_implementation("Actor").__init__(self, context)

    def terminate(self):
        self.stop()


class ServiceDiscovery:
    def __init__(self, service, history_limit=0):
        self.services_cache = services_cache_create_singleton(service, history_limit=history_limit)

    def add_handler(self, service_change_handler, filter):
        self.services_cache.add_handler(service_change_handler, filter)

    def remove_handler(self, service_change_handler, filter):
        self.services_cache.remove_handler(service_change_handler, filter)

    def get_services(self, filter=None):
        services = self.services_cache.get_services()
        return services if filter is None else services.filter_services(filter)


class ActorDiscovery(ServiceDiscovery):
    def get_actor_mqtt(self, filter, protocol_class):
        """Proxy for the first discovered service matching ``filter`` (None if none yet)."""
        for details in self.get_services(filter):
            return get_actor_mqtt(f"{details[0] if not isinstance(details, dict) else details['topic_path']}/in",
                                  protocol_class)
        return None


def get_public_methods(protocol_class):
    if isinstance(protocol_class, str):
        raise ValueError(f"{protocol_class} is a String, should be a Class reference ?")
    names = [n for n, _ in getmembers(protocol_class, isfunction) if not n.startswith("_")]
    if not names:
        raise ValueError(f"Class {protocol_class} has no public methods")
    return names


class ServiceRemoteProxy:
    """Attributes are publishers; ``topic_in`` names the remote actor."""

    def __init__(self, topic_in):
        self.topic_in = topic_in

    def __repr__(self):
        return f"ServiceRemoteProxy({self.topic_in})"


def make_proxy_mqtt(target_topic_in, public_method_names):
    proxy = ServiceRemoteProxy(target_topic_in)

    def sender(method_name):
        def closure(*args, **kwargs):
            parameters = list(args)
            if kwargs:
                parameters.append(kwargs)
            # arrays (tensors, ndarrays, DeviceResults) travel as one binary payload
            aiko.message.publish(target_topic_in, encode_message(method_name, parameters))
        closure.__name__ = method_name
        return closure

    for name in public_method_names:
        setattr(proxy, name, sender(name))
    return proxy


def get_actor_mqtt(target_service_topic_in, protocol_class):
    return make_proxy_mqtt(target_service_topic_in, get_public_methods(protocol_class))
