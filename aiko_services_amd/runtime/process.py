"""Process runtime: the ``aiko`` singleton (reference ``main/process.py:76-355``).

``aiko`` (= :class:`ProcessData`) carries the process topic paths
``{namespace}/{hostname}/{pid}/0/{in,log,state,out}``, the transport (``aiko.message``), the
connection state, the discovered registrar and the logger factory.  ``aiko.process`` is the
:class:`ProcessImplementation` singleton that owns the topic -> handler table, the service
table, the registrar boot handshake and the event loop.

Differences from the reference (bugs fixed): wildcard topics are matched
with a real MQTT topic trie (``+`` any level, ``#`` any suffix); ``remove_service`` and binary
topic removal work; handler exceptions are logged to the process log topic and never kill the
loop.  Inbound transport messages are queued onto the event loop (one thread runs all actor
code), and the loop drains every queued message per wakeup.
"""
from __future__ import annotations

import os
import sys
import threading
import traceback

from ..message import MQTT, Castaway
from ..message.mqtt_codec import TopicTrie
from ..utils.configuration import get_hostname, get_namespace, get_pid, get_username
from ..utils.logger import DEBUG, LoggingHandlerMQTT, get_logger
from ..utils.misc import ContextManager, Lock
from ..message.tensor_payload import encode_message, is_tensor_payload
from ..utils.sexpr import generate, parse
from . import event
from .connection import Connection, ConnectionState

__all__ = ["aiko", "process_create", "ProcessData", "ProcessImplementation"]


class ProcessData:
    TOPIC_REGISTRAR_BOOT = f"{get_namespace()}/service/registrar"

    connection = Connection()
    logger = None
    message = None
    process = None
    registrar = None

    topic_path_process = f"{get_namespace()}/{get_hostname()}/{get_pid()}"
    topic_path = f"{topic_path_process}/0"
    topic_in = f"{topic_path}/in"
    topic_log = f"{topic_path}/log"
    topic_lwt = f"{topic_path}/state"
    topic_out = f"{topic_path}/out"
    payload_lwt = "(absent)"

    @classmethod
    def get_topic_path(cls, service_id):
        return f"{cls.topic_path_process}/{service_id}"


aiko = ProcessData


class AikoLogger:
    @classmethod
    def logger(cls, name, log_level=None, logging_handler=None, topic=None):
        if logging_handler is None:
            option = os.environ.get("AIKO_LOG_MQTT", "all")
            if option in ("all", "true"):
                logging_handler = LoggingHandlerMQTT(aiko, topic or aiko.topic_log, option)
        return get_logger(name, log_level, logging_handler)


aiko.logger = AikoLogger.logger

_LOGGER_MESSAGE = aiko.logger(f"{__name__}.message",
                              log_level=os.environ.get("AIKO_LOG_LEVEL_MESSAGE", "INFO"))
_LOGGER = aiko.logger(__name__, log_level=os.environ.get("AIKO_LOG_LEVEL_PROCESS", "INFO"))


class ProcessImplementation(ProcessData):
    def __init__(self):
        self.initialized = False
        self.running = False
        self.service_count = 0
        self._service_id_next = 0
        self._exit_status = 0
        self._message_handlers: dict = {}        # topic -> [handler]
        self._binary_topics: set = set()
        self._wildcards = TopicTrie()
        self._wildcard_topics: set = set()
        self._registrar_absent_terminate = False
        self._services: dict = {}
        self._services_lock = Lock(f"{__name__}._services", _LOGGER)
        self.message_count = 0

    # ---- lifecycle ------------------------------------------------------------------------
    def initialize(self, mqtt_connection_required=True, message=None):
        """Connect the transport.  ``message`` injects a transport (e.g. ``Loopback``)."""
        if self.initialized:
            return
        self.initialized = True
        event.add_queue_handler(self.on_message_queue_handler, ["message"])
        self.add_message_handler(self.on_registrar, aiko.TOPIC_REGISTRAR_BOOT)
        if message is not None:
            aiko.message = message
            message.message_handler = self.on_message
            message.set_last_will_and_testament(aiko.topic_lwt, aiko.payload_lwt, False)
            message.subscribe(list(self._message_handlers))
            aiko.connection.update_state(ConnectionState.TRANSPORT)
        else:
            aiko.message = Castaway()
            connected = False
            if os.environ.get("AIKO_MQTT_DISABLE", "") not in ("1", "true"):
                try:
                    aiko.message = MQTT(self.on_message, self._message_handlers,
                                        aiko.topic_lwt, aiko.payload_lwt, False)
                    connected = True
                except SystemError as exc:
                    (_LOGGER.error if mqtt_connection_required else _LOGGER.debug)(exc)
            if mqtt_connection_required and not connected:
                raise SystemExit(1)
            if connected:
                aiko.connection.update_state(ConnectionState.TRANSPORT)
        ContextManager(aiko, aiko.message)

    def run(self, loop_when_no_handlers=False, mqtt_connection_required=True):
        self.initialize(mqtt_connection_required=mqtt_connection_required)
        if not self.running:
            try:
                self.running = True
                event.loop(loop_when_no_handlers)
            finally:
                self.running = False
        if self._exit_status:
            sys.exit(self._exit_status)

    def run_in_thread(self, loop_when_no_handlers=True, mqtt_connection_required=False, message=None):
        """Start the event loop on a daemon thread (embedding / tests)."""
        self.initialize(mqtt_connection_required=mqtt_connection_required, message=message)
        t = threading.Thread(target=self.run, args=(loop_when_no_handlers, mqtt_connection_required),
                             name="aiko-event-loop", daemon=True)
        t.start()
        return t

    def terminate(self, exit_status=0):
        self._exit_status = exit_status
        event.terminate()

    def set_last_will_and_testament(self, topic_lwt, payload_lwt="(absent)", retain_lwt=False):
        aiko.message.set_last_will_and_testament(topic_lwt, payload_lwt, retain_lwt)

    def set_registrar_absent_terminate(self):
        self._registrar_absent_terminate = True

    # ---- topic routing ----------------------------------------------------------------------
    def add_message_handler(self, message_handler, topic, binary=False):
        if topic not in self._message_handlers:
            self._message_handlers[topic] = []
            if binary:
                self._binary_topics.add(topic)
            if "#" in topic or "+" in topic:
                self._wildcard_topics.add(topic)
                self._wildcards.add(topic, topic)
            if aiko.message is not None:
                aiko.message.subscribe(topic)
        self._message_handlers[topic].append(message_handler)

    def remove_message_handler(self, message_handler, topic):
        handlers = self._message_handlers.get(topic)
        if handlers is None:
            return
        if message_handler in handlers:
            handlers.remove(message_handler)
        if not handlers:
            del self._message_handlers[topic]
            self._binary_topics.discard(topic)
            if topic in self._wildcard_topics:
                self._wildcard_topics.discard(topic)
                self._wildcards.remove(topic, topic)
            if aiko.message is not None:
                aiko.message.unsubscribe(topic)

    def topic_matcher(self, topic, topics=None):
        matched = [topic] if topic in self._message_handlers else []
        if self._wildcard_topics:
            matched.extend(t for t in self._wildcards.match(topic) if t != topic)
        return matched

    def on_message(self, client, userdata, message):
        event.queue_put(message, "message")

    def on_message_queue_handler(self, message, _item_type):
        topic = message.topic
        payload = message.payload
        self.message_count += 1
        handlers = []
        binary = False
        for t in self.topic_matcher(topic):
            handlers.extend(self._message_handlers.get(t, ()))
            binary = binary or t in self._binary_topics
        if not binary and isinstance(payload, (bytes, bytearray)) and not is_tensor_payload(payload):
            # (a tensor payload stays bytes: parse() decodes it, arrays included)
            try:
                payload = payload.decode("utf-8")
            except UnicodeDecodeError:
                _LOGGER.warning(f"non UTF-8 payload on text topic {topic}")
                return
        if _LOGGER_MESSAGE.isEnabledFor(DEBUG):
            _LOGGER_MESSAGE.debug(f"Message: {topic}: {payload}")
        for handler in handlers:
            try:
                if handler(aiko, topic, payload):
                    return
            except SystemExit:
                raise
            except Exception:
                trace = traceback.format_exc()
                print(trace, file=sys.stderr)
                try:
                    aiko.message.publish(aiko.topic_log, trace)
                except Exception:
                    pass

    # ---- services -----------------------------------------------------------------------------
    def _add_service_to_registrar(self, service):
        if service.protocol and aiko.registrar:
            tags = service.get_tags_string()
            payload = (f"(add {service.topic_path} {service.name} {service.protocol} "
                       f"{service.transport} {get_username()} ({tags}))")
            aiko.message.publish(f"{aiko.registrar['topic_path']}/in", payload)

    def _remove_service_from_registrar(self, service):
        if service.protocol and aiko.registrar:
            aiko.message.publish(f"{aiko.registrar['topic_path']}/in", f"(remove {service.topic_path})")

    def add_service(self, service):
        self._services_lock.acquire("add_service()")
        try:
            self._service_id_next += 1
            self.service_count += 1
            service.service_id = self._service_id_next
            service.topic_path = aiko.get_topic_path(service.service_id)
            self._services[service.service_id] = service
        finally:
            self._services_lock.release()
        if aiko.connection.is_connected(ConnectionState.REGISTRAR):
            self._add_service_to_registrar(service)
        return service.service_id

    def remove_service(self, service_id):
        self._services_lock.acquire("remove_service()")
        try:
            service = self._services.pop(service_id, None)
            if service is not None:
                self.service_count -= 1
        finally:
            self._services_lock.release()
        if service is not None and aiko.connection.is_connected(ConnectionState.REGISTRAR):
            self._remove_service_from_registrar(service)
        return self.service_count

    def get_service(self, service_id):
        return self._services.get(service_id)

    def services(self):
        return list(self._services.values())

    # ---- registrar boot handshake (retained "(primary found ...)") ----------------------------
    def on_registrar(self, _aiko, topic, payload_in):
        try:
            command, parameters = parse(payload_in)
        except Exception:
            return
        if command != "primary" or not parameters:
            return
        action = parameters[0]
        if action == "found" and len(parameters) == 4:
            aiko.registrar = {"topic_path": parameters[1], "version": parameters[2],
                              "timestamp": parameters[3]}
            aiko.connection.update_state(ConnectionState.REGISTRAR)
            for service in list(self._services.values()):
                self._add_service_to_registrar(service)
        elif action == "absent" and len(parameters) == 1:
            aiko.registrar = None
            aiko.connection.update_state(ConnectionState.TRANSPORT)
            if self._registrar_absent_terminate:
                self.terminate(1)
        else:
            return
        for service in list(self._services.values()):
            service.registrar_handler_call(action, aiko.registrar)


def process_create():
    if not ProcessData.process:
        ProcessData.process = ProcessImplementation()
    return ProcessData.process


def publish_generate(topic, command, parameters, retain=False):
    """Convenience: publish ``generate(command, parameters)`` on ``topic``."""
    aiko.message.publish(topic, encode_message(command, parameters), retain=retain)
