"""Services: discoverable components with topic paths, protocol and tags.

Reference ``main/service.py:105-583``: ``ServiceProtocol``, ``ServiceFields``,
``ServiceFilter``, ``ServiceTags``, ``ServiceTopicPath``, ``Services`` (2-level
process -> service table with attribute filtering), ``Service`` interface and ``ServiceImpl``.
"""
from __future__ import annotations

import time
from abc import abstractmethod

from .context import Interface, ServiceProtocolInterface
from .process import aiko

__all__ = ["ServiceFields", "ServiceFilter", "ServiceProtocol", "ServiceTags", "ServiceTopicPath",
           "Services", "Service", "ServiceImpl"]


class ServiceProtocol:
    AIKO = "github.com/geekscape/aiko_services/protocol"

    def __init__(self, url_prefix, name, version):
        self.url_prefix = url_prefix
        self.name = name
        self.version = version

    def __repr__(self):
        return f"{self.url_prefix}/{self.name}:{self.version}"


class ServiceFields:
    def __init__(self, topic_path, name, protocol, transport, owner, tags):
        self.topic_path = topic_path
        self.name = name
        self.protocol = protocol
        self.transport = transport
        self.owner = owner
        self.tags = tags

    def __repr__(self):
        return (f"{self.topic_path}, {self.name}, {self.protocol}, {self.transport}, "
                f"{self.owner}, {self.tags}")


class ServiceFilter:
    @classmethod
    def with_topic_path(cls, topic_path="*", name="*", protocol="*", transport="*", owner="*",
                        tags="*"):
        topic_paths = topic_path if topic_path == "*" else [topic_path]
        return ServiceFilter(topic_paths, name, protocol, transport, owner, tags)

    def __init__(self, topic_paths="*", name="*", protocol="*", transport="*", owner="*", tags="*"):
        self.topic_paths = topic_paths
        self.name = name
        self.protocol = protocol
        self.transport = transport
        self.owner = owner
        self.tags = tags

    def __repr__(self):
        return (f"{self.topic_paths}, {self.name}, {self.protocol}, {self.transport}, "
                f"{self.owner}, {self.tags}")

    def matches(self, details) -> bool:
        name, protocol, transport, owner, tags = _fields(details)
        if self.name != "*" and self.name != name:
            return False
        if self.protocol != "*" and self.protocol != protocol:
            return False
        if self.transport != "*" and self.transport != transport:
            return False
        if self.owner != "*" and self.owner != owner:
            return False
        if self.tags != "*":
            want = self.tags if isinstance(self.tags, list) else [self.tags]
            if not ServiceTags.match_tags(tags, want):
                return False
        return True


class ServiceTags:
    @classmethod
    def get_tag_value(cls, key, tags):
        return ServiceTags.parse_tags(tags).get(key)

    @classmethod
    def match_tags(cls, service_tags, match_tags):
        return all(tag in service_tags for tag in match_tags)

    @classmethod
    def parse_tags(cls, tags_list):
        tags = {}
        for tag in tags_list:
            key, _, value = tag.partition("=")
            tags[key] = value
        return tags


class ServiceTopicPath:
    @classmethod
    def parse(cls, topic_path):
        parts = topic_path.split("/") if isinstance(topic_path, str) else []
        if len(parts) != 4:
            return None
        return ServiceTopicPath(*parts)

    @classmethod
    def topic_paths(cls, topic_path):
        stp = ServiceTopicPath.parse(topic_path)
        return (stp.topic_path_process if stp else None), str(stp)

    def __init__(self, namespace, hostname, process_id=0, service_id=0):
        self.namespace = namespace
        self.hostname = hostname
        self.process_id = process_id
        self.service_id = service_id

    def __repr__(self):
        return f"{self.topic_path_process}/{self.service_id}"

    @property
    def terse(self):
        topic_path = str(self)
        if len(topic_path) > 26:
            namespace = self.namespace[0:4] + ("+" if len(self.namespace) > 4 else "")
            hostname = self.hostname[0:8] + ("+" if len(self.hostname) > 8 else "")
            topic_path = f"{namespace}/{hostname}/{self.process_id}/{self.service_id}"
        return topic_path

    @property
    def topic_path_process(self):
        return f"{self.namespace}/{self.hostname}/{self.process_id}"


def _fields(details):
    """(name, protocol, transport, owner, tags) from a dict or a positional list."""
    if isinstance(details, dict):
        return details["name"], details["protocol"], details["transport"], details["owner"], details["tags"]
    return details[1], details[2], details[3], details[4], details[5]


class Services:
    """process topic path -> {service topic path -> details}."""

    def __init__(self):
        self._count = 0
        self._services: dict = {}

    def __iter__(self):
        for process_services in list(self._services.values()):
            yield from list(process_services.values())

    def __len__(self):
        return self._count

    def __str__(self):
        return "\n".join(self.get_topic_paths())

    def add_service(self, topic_path, service_details):
        process_tp, service_tp = ServiceTopicPath.topic_paths(topic_path)
        if process_tp:
            ps = self._services.setdefault(process_tp, {})
            if service_tp not in ps:
                ps[service_tp] = service_details
                self._count += 1

    def copy(self):
        clone = Services()
        clone._services = {k: dict(v) for k, v in self._services.items()}
        clone._count = self._count
        return clone

    @property
    def count(self):
        return self._count

    def filter_services(self, filter):
        return self.filter_by_attributes(filter, services=self.filter_by_topic_paths(filter.topic_paths))

    def filter_by_attributes(self, filter, services=None):
        source = services._services if services is not None else self._services
        results = Services()
        for process_services in source.values():
            for topic, details in process_services.items():
                if filter.matches(details):
                    results.add_service(topic, details)
        return results

    def filter_by_topic_paths(self, topic_paths):
        if topic_paths == "*":
            return self
        results = Services()
        for tp in topic_paths:
            process_tp, _ = ServiceTopicPath.topic_paths(tp)
            ps = self._services.get(process_tp)
            if ps and tp in ps:
                results.add_service(tp, ps[tp])
        return results

    def get_process_services(self, process_topic_path):
        ps = self._services.get(process_topic_path)
        return list(ps.keys()) if ps else []

    def get_service(self, topic_path):
        process_tp, service_tp = ServiceTopicPath.topic_paths(topic_path)
        ps = self._services.get(process_tp)
        return ps.get(service_tp) if ps else None

    def get_topic_paths(self):
        out = []
        for ps in self._services.values():
            out.extend(ps.keys())
        return out

    def remove_service(self, topic_path):
        process_tp, service_tp = ServiceTopicPath.topic_paths(topic_path)
        ps = self._services.get(process_tp)
        if ps is None:
            return
        if service_tp in ps:
            del ps[service_tp]
            self._count -= 1
        if not ps:
            del self._services[process_tp]


class Service(ServiceProtocolInterface):
    Interface.default("Service", "aiko_services_amd.runtime.service.ServiceImpl")

    @abstractmethod
    def add_message_handler(self, message_handler, topic, binary=False):
        pass

    @abstractmethod
    def remove_message_handler(self, message_handler, topic):
        pass

    @abstractmethod
    def registrar_handler_call(self, action, registrar):
        pass

    @abstractmethod
    def run(self):
        pass

    @abstractmethod
    def set_registrar_handler(self, registrar_handler):
        pass

    @abstractmethod
    def stop(self):
        pass

    @abstractmethod
    def add_tags(self, tags):
        pass

    @abstractmethod
    def add_tags_string(self, tags_string):
        pass

    @abstractmethod
    def get_tags_string(self):
        pass


class ServiceImpl(Service):
    def __init__(self, context):
        self.time_started = time.time()
        self.name = context.name
        self.protocol = context.protocol
        self._tags = context.tags
        self.transport = context.transport
        aiko.process.add_service(self)   # sets service_id and topic_path
        self._registrar_handler_function = None
        self.topic_control = f"{self.topic_path}/control"
        self.topic_in = f"{self.topic_path}/in"
        self.topic_log = f"{self.topic_path}/log"
        self.topic_out = f"{self.topic_path}/out"
        self.topic_state = f"{self.topic_path}/state"

    def add_message_handler(self, message_handler, topic, binary=False):
        aiko.process.add_message_handler(message_handler, topic, binary)

    def remove_message_handler(self, message_handler, topic):
        aiko.process.remove_message_handler(message_handler, topic)

    def registrar_handler_call(self, action, registrar):
        if self._registrar_handler_function:
            self._registrar_handler_function(action, registrar)

    def run(self):
        aiko.process.run()

    def set_registrar_handler(self, registrar_handler):
        self._registrar_handler_function = registrar_handler

    def stop(self):
        aiko.process.terminate()

    def add_tags(self, tags):
        for tag in tags:
            if not ServiceTags.match_tags(self._tags, [tag]):
                self._tags.append(tag)

    def add_tags_string(self, tags_string):
        if tags_string:
            self.add_tags(tags_string.split(","))

    def get_tags_string(self):
        return " ".join(str(tag) for tag in self._tags)

    @property
    def tags(self):
        return self._tags
