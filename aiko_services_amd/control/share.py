"""Eventually-consistent shared state: ECProducer / ECConsumer and the ServicesCache.

Reference ``main/share.py:93-656``; wire protocol unchanged:

* consumer -> producer ``{svc}/control``: ``(share <response_topic> <lease_time> <filter>)``,
  ``lease_time 0`` cancels (or requests a one-shot sync);
* producer -> consumer: ``(item_count N)`` then N x ``(add name value)``, then live
  ``(add|update|remove ...)``; producer echoes changes and ``(sync <topic>)`` on ``{svc}/state``;
* anyone -> producer ``(add|update|remove name [value])`` edits the share (dashboard edits).

Shares are dictionaries of depth <= 2 (``"a.b"`` item names).  Unlike the reference, update
values are S-expression encoded (values with spaces survive), and ServicesCache is the
client-side replica of the registrar (``empty -> history -> share -> loaded -> ready``).
"""
from __future__ import annotations

import threading
import time
from collections import deque

from ..runtime import event
from ..runtime.connection import ConnectionState
from ..runtime.lease import Lease
from ..runtime.process import aiko
from ..runtime.service import ServiceProtocol, Services
from ..utils.sexpr import generate, parse, parse_int

__all__ = ["ECConsumer", "ECProducer", "PROTOCOL_EC_CONSUMER", "PROTOCOL_EC_PRODUCER",
           "ServicesCache", "services_cache_create_singleton", "services_cache_delete",
           "services_cache_get"]

_VERSION = 0
PROTOCOL_EC_CONSUMER = f"{ServiceProtocol.AIKO}/ec_consumer_test:{_VERSION}"
PROTOCOL_EC_PRODUCER = f"{ServiceProtocol.AIKO}/ec_producer_test:{_VERSION}"
LEASE_TIME = 300
HISTORY_RING_BUFFER_SIZE = 4096

_LOGGER = None


def _logger():
    global _LOGGER
    if _LOGGER is None:
        import os
        _LOGGER = aiko.logger(__name__, log_level=os.environ.get("AIKO_LOG_LEVEL_SHARE", "INFO"))
    return _LOGGER


# ---- item helpers ---------------------------------------------------------------------------

def _parse_item_path(name):
    path = str(name).split(".")
    if len(path) > 2:
        raise ValueError(f'EC "share" dictionary depth maximum is 2: {name}')
    return path


def _modify(items, path, op, create=False):
    if not isinstance(items, dict):
        raise ValueError(f'"items" must be a dictionary, not {type(items).__name__}')
    if not path:
        raise ValueError('"item_path" must be non-empty')
    key, *tail = path
    if not tail:
        op(items, key)
    elif key in items:
        _modify(items[key], tail, op, create)
    elif create:
        items[key] = {}
        _modify(items[key], tail, op, create)


def _update_item(share, path, value):
    def op(items, key):
        items[key] = value
    _modify(share, path, op, create=True)


def _remove_item(share, path):
    def op(items, key):
        items.pop(key, None)
    _modify(share, path, op)


def _flatten(d):
    out = []
    for name, item in d.items():
        if isinstance(item, dict):
            for sub, v in item.items():
                out.append((f"{name}.{sub}", v))
        else:
            out.append((name, item))
    return out


def _filter_compare(filter_, item_name) -> bool:
    if filter_ == "*":
        return True
    return any(item_name == f or item_name.startswith(f"{f}.") for f in filter_)


class ECLease(Lease):
    def __init__(self, lease_time, topic, filter=None, lease_expired_handler=None):
        super().__init__(lease_time, topic, lease_expired_handler=lease_expired_handler)
        self.filter = filter


class ECProducer:
    def __init__(self, service, share, topic_in=None, topic_out=None):
        self.share = share
        self.topic_in = topic_in or service.topic_control
        self.topic_out = topic_out or service.topic_state
        self.handlers: list = []
        self.leases: dict = {}
        service.add_message_handler(self._producer_handler, self.topic_in)
        service.add_tags(["ec=true"])

    def add_handler(self, handler):
        for name, value in _flatten(self.share):
            handler("add", name, value)
        if handler not in self.handlers:
            self.handlers.append(handler)

    def remove_handler(self, handler):
        if handler in self.handlers:
            self.handlers.remove(handler)

    def get(self, item_name):
        item = self.share
        for key in _parse_item_path(item_name):
            if isinstance(item, dict) and key in item:
                item = item[key]
            else:
                return None
        return item

    def update(self, item_name, item_value):
        try:
            _update_item(self.share, _parse_item_path(item_name), item_value)
        except ValueError as exc:
            _logger().error(f"update(): {item_name}: {exc}")
            return
        self._update_consumers("update", item_name, item_value)

    def remove(self, item_name):
        try:
            _remove_item(self.share, _parse_item_path(item_name))
        except ValueError as exc:
            _logger().error(f"remove(): {item_name}: {exc}")
            return
        self._update_consumers("remove", item_name, None)

    def _producer_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command in ("add", "update") and len(parameters) == 2:
            name, value = parameters
            try:
                _update_item(self.share, _parse_item_path(name), value)
            except ValueError as exc:
                _logger().error(f"_producer_handler(): {command} {parameters}: {exc}")
                return
            aiko.message.publish(self.topic_out, payload_in)
            self._update_consumers(command, name, value)
        elif command == "remove" and len(parameters) == 1:
            name = parameters[0]
            try:
                _remove_item(self.share, _parse_item_path(name))
            except ValueError as exc:
                _logger().error(f"_producer_handler(): {command} {parameters}: {exc}")
                return
            aiko.message.publish(self.topic_out, payload_in)
            self._update_consumers(command, name, None)
        elif command == "share" and len(parameters) == 3:
            response_topic = parameters[0]
            try:
                lease_time = int(parameters[1])
            except (TypeError, ValueError):
                return
            filter_ = parameters[2]
            if filter_ != "*" and not isinstance(filter_, list):
                filter_ = [filter_]
            if lease_time == 0:
                lease = self.leases.pop(response_topic, None)
                if lease is not None:
                    lease.terminate()
                else:
                    self._synchronize(response_topic, filter_)
            elif lease_time > 0:
                lease = self.leases.get(response_topic)
                if lease is not None:
                    lease.extend(lease_time)
                else:
                    self.leases[response_topic] = ECLease(lease_time, response_topic, filter_,
                                                          self._lease_expired_handler)
                    self._synchronize(response_topic, filter_)

    def _lease_expired_handler(self, topic):
        self.leases.pop(topic, None)

    def _filter_dictionary(self, d, filter_, path):
        out = {}
        for name, item in d.items():
            item_path = path + [str(name)]
            if isinstance(item, dict):
                sub = self._filter_dictionary(item, filter_, item_path)
                if sub:
                    out[name] = sub
            elif _filter_compare(filter_, ".".join(item_path)):
                out[name] = item
        return out

    def _synchronize(self, response_topic, filter_):
        commands = [generate("add", [name, value])
                    for name, value in _flatten(self._filter_dictionary(self.share, filter_, []))]
        aiko.message.publish(response_topic, f"(item_count {len(commands)})")
        for payload in commands:
            aiko.message.publish(response_topic, payload)
        aiko.message.publish(self.topic_out, f"(sync {response_topic})")

    def _update_consumers(self, command, item_name, item_value):
        for handler in list(self.handlers):
            handler(command, item_name, item_value)
        if not self.leases:
            return
        if command == "remove":
            payload = generate(command, [item_name])
        else:
            payload = generate(command, [item_name, item_value])
        for lease in list(self.leases.values()):
            if _filter_compare(lease.filter, item_name):
                aiko.message.publish(lease.lease_uuid, payload)


class ECConsumer:
    """Leased replica of a remote ECProducer's share (``cache`` is updated in place)."""

    def __init__(self, service, ec_consumer_id, cache, ec_producer_topic_control, filter="*"):
        self.service = service
        self.ec_consumer_id = ec_consumer_id
        self.cache = cache
        self.ec_producer_topic_control = ec_producer_topic_control
        self.filter = filter
        self.cache_state = "empty"
        self.handlers: list = []
        self.item_count = 0
        self.items_received = 0
        self.lease = None
        self.topic_share_in = f"{service.topic_path}/{ec_producer_topic_control}/{ec_consumer_id}/in"
        service.add_message_handler(self._consumer_handler, self.topic_share_in)
        aiko.connection.add_handler(self._connection_state_handler)

    def add_handler(self, handler):
        for name, value in _flatten(self.cache):
            handler(self.ec_consumer_id, "add", name, value)
        if handler not in self.handlers:
            self.handlers.append(handler)

    def remove_handler(self, handler):
        if handler in self.handlers:
            self.handlers.remove(handler)

    def _consumer_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command == "item_count" and len(parameters) == 1:
            self.item_count = parse_int(parameters[0])
            self.items_received = 0
            if self.item_count == 0:
                self.cache_state = "ready"
        elif command in ("add", "update") and len(parameters) == 2:
            name, value = parameters
            try:
                _update_item(self.cache, _parse_item_path(name), value)
            except ValueError as exc:
                _logger().warning(f"ECConsumer: {command} {name}: {exc}")
                return
            if command == "add":
                self.items_received += 1
                if self.items_received == self.item_count:
                    self.cache_state = "ready"
            self._update_handlers(command, name, value)
        elif command == "remove" and len(parameters) == 1:
            name = parameters[0]
            try:
                _remove_item(self.cache, _parse_item_path(name))
            except ValueError as exc:
                _logger().warning(f"ECConsumer: remove {name}: {exc}")
                return
            self._update_handlers(command, name, None)
        elif command == "sync":
            self._update_handlers(command, None, None)

    def _connection_state_handler(self, connection, connection_state):
        if connection.is_connected(ConnectionState.REGISTRAR) and not self.lease:
            self.lease = Lease(LEASE_TIME, None, automatic_extend=True,
                               lease_extend_handler=self._share_request)
            self._share_request()

    def _share_request(self, lease_time=LEASE_TIME, lease_uuid=None):
        filter_ = self.filter
        if isinstance(filter_, (list, tuple)):
            filter_ = generate(filter_[0], list(filter_[1:])) if filter_ else "*"
        aiko.message.publish(self.ec_producer_topic_control,
                             f"(share {self.topic_share_in} {lease_time} {filter_})")

    def _update_handlers(self, command, name, value):
        for handler in list(self.handlers):
            handler(self.ec_consumer_id, command, name, value)

    def terminate(self):
        self.service.remove_message_handler(self._consumer_handler, self.topic_share_in)
        aiko.connection.remove_handler(self._connection_state_handler)
        self.cache = {}
        self.cache_state = "empty"
        if self.lease:
            self.lease.terminate()
            self.lease = None
            self._share_request(lease_time=0)


# ---- ServicesCache ---------------------------------------------------------------------------

class ServicesCache:
    def __init__(self, service, event_loop_start=False, history_limit=0):
        self._service = service
        self._event_loop_start = event_loop_start
        self._event_loop_owner = False
        self._history_limit = history_limit
        self._handlers: list = []
        self._history: deque = deque(maxlen=HISTORY_RING_BUFFER_SIZE)
        self._registrar_topic_share = f"{service.topic_path}/registrar_share"
        self._ready = threading.Event()
        self._cache_reset()
        aiko.connection.add_handler(self._connection_state_handler)

    def _cache_reset(self):
        self._begin_registration = False
        self._item_count = None
        self._registrar_service = None
        self._registrar_topic_in = None
        self._registrar_topic_out = None
        self._services = Services()
        self._state = "empty"
        self._ready.clear()

    def add_handler(self, service_change_handler, service_filter):
        if self._state in ("loaded", "ready"):
            service_change_handler("sync", None)
            for details in self._services.filter_services(service_filter):
                service_change_handler("add", details)
        self._handlers.append((service_change_handler, service_filter))

    def remove_handler(self, service_change_handler, service_filter):
        entry = (service_change_handler, service_filter)
        if entry in self._handlers:
            self._handlers.remove(entry)

    def _connection_state_handler(self, connection, connection_state):
        if connection.is_connected(ConnectionState.REGISTRAR):
            if not self._begin_registration:
                self._begin_registration = True
                topic_path = aiko.registrar["topic_path"]
                self._registrar_topic_in = f"{topic_path}/in"
                self._registrar_topic_out = f"{topic_path}/out"
                self._service.add_message_handler(self.registrar_out_handler, self._registrar_topic_out)
                self._service.add_message_handler(self.registrar_share_handler, self._registrar_topic_share)
                if self._history_limit > 0:
                    self._state = "history"
                    aiko.message.publish(self._registrar_topic_in,
                                         f"(history {self._registrar_topic_share} {self._history_limit})")
                else:
                    self._state = "share"
                    self._publish_registrar_share()
        elif self._registrar_topic_out:
            self._service.remove_message_handler(self.registrar_out_handler, self._registrar_topic_out)
            self._service.remove_message_handler(self.registrar_share_handler, self._registrar_topic_share)
            if self._registrar_service:
                self._history.appendleft(self._registrar_service)
            self._cache_reset()

    def _publish_registrar_share(self):
        aiko.message.publish(self._registrar_topic_in, f"(share {self._registrar_topic_share} * * * * *)")

    def _update_handlers(self, command, details=None):
        topic_path = details[0] if details else None
        for handler, filter_ in list(self._handlers):
            if topic_path:
                if filter_.topic_paths != "*" and topic_path not in filter_.topic_paths:
                    continue
                if not filter_.matches(details):
                    continue
            handler(command, details)

    def get_history(self):
        return self._history

    def get_services(self):
        return self._services

    def get_state(self):
        return self._state

    def registrar_share_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command == "item_count" and len(parameters) == 1:
            self._item_count = int(parameters[0])
        elif command == "add" and len(parameters) >= 6 and self._item_count is not None:
            self._item_count -= 1
            if self._state == "history":
                self._history.append(parameters)
            elif self._state == "share":
                self._services.add_service(parameters[0], parameters)
                if aiko.registrar and parameters[0] == aiko.registrar["topic_path"]:
                    self._registrar_service = parameters
        if self._item_count == 0:
            self._item_count = None
            if self._state == "history":
                self._state = "share"
                self._publish_registrar_share()
            elif self._state == "share":
                self._state = "loaded"
                self._update_handlers("sync")
                for details in self._services:
                    self._update_handlers("add", details)

    def registrar_out_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command == "sync" and len(parameters) == 1:
            if parameters[0] == self._registrar_topic_share and self._state == "loaded":
                self._state = "ready"
                self._ready.set()
        elif command == "add" and len(parameters) == 6:
            self._services.add_service(parameters[0], parameters)
            self._update_handlers(command, parameters)
        elif command == "remove" and parameters:
            details = self._services.get_service(parameters[0])
            if details:
                self._update_handlers(command, details)
                self._services.remove_service(parameters[0])
                self._history.appendleft(details)

    def run(self):
        if self._event_loop_start and not event.is_running():
            self._event_loop_owner = True
            aiko.process.run()

    def terminate(self):
        if self._event_loop_owner:
            aiko.process.terminate()

    def wait_ready(self, timeout=None):
        return self._ready.wait(timeout)


_services_cache = None


def services_cache_create_singleton(service, event_loop_start=False, history_limit=0):
    global _services_cache
    if _services_cache is None:
        _services_cache = ServicesCache(service, event_loop_start, history_limit)
        if event_loop_start:
            threading.Thread(target=_services_cache.run, daemon=True).start()
    return _services_cache


def services_cache_get():
    return _services_cache


def services_cache_delete():
    global _services_cache
    if _services_cache is not None:
        _services_cache.terminate()
        _services_cache = None
