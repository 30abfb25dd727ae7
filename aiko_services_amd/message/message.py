"""Control-plane transports: ``Message`` ABC, ``Castaway`` (null), ``Loopback`` (in-process bus)
and ``MQTT`` (network, own client).

Reference: ``main/message/{message,castaway,mqtt}.py``.  Every transport delivers inbound
messages by calling ``message_handler(client, userdata, message)`` with a message exposing
``.topic`` and ``.payload`` (bytes) — the process queues it onto the event loop.

``Loopback`` is a process-local broker with MQTT semantics (wildcards, retained messages,
last-will on ``simulate_disconnect``); several ``Loopback`` endpoints may share one
``LoopbackBus`` to emulate several processes in a single test process.
"""
from __future__ import annotations

import os
import threading
import time
from abc import ABC, abstractmethod

from ..utils import fault as _fault
from ..utils.configuration import get_mqtt_configuration
from . import mqtt_codec as C
from .mqtt_client import MQTTClient, MQTTMessage
from .websocket import is_websocket_transport

__all__ = ["Message", "Castaway", "Loopback", "LoopbackBus", "MQTT"]


class Message(ABC):
    @abstractmethod
    def publish(self, topic, payload, retain=False, wait=False):
        ...

    @abstractmethod
    def subscribe(self, topics):
        ...

    @abstractmethod
    def unsubscribe(self, topics):
        ...

    @abstractmethod
    def set_last_will_and_testament(self, topic_lwt, payload_lwt="(absent)", retain_lwt=False):
        ...

    def terminate(self):
        pass

    def is_connected(self) -> bool:
        return False


class Castaway(Message):
    """Standalone and isolated: publishes go nowhere (reference ``castaway.py``)."""

    def __init__(self, *args, **kwargs):
        self.published = 0

    def publish(self, topic, payload, retain=False, wait=False):
        self.published += 1

    def subscribe(self, topics):
        pass

    def unsubscribe(self, topics):
        pass

    def set_last_will_and_testament(self, topic_lwt, payload_lwt="(absent)", retain_lwt=False):
        pass


class LoopbackBus:
    """A tiny in-process broker shared by ``Loopback`` endpoints."""

    def __init__(self):
        self.lock = threading.RLock()
        self.trie = C.TopicTrie()
        self.retained: dict = {}
        self.endpoints: list = []

    def route(self, topic, payload: bytes, retain: bool):
        with self.lock:
            if retain:
                if payload:
                    self.retained[topic] = payload
                else:
                    self.retained.pop(topic, None)
            targets = list(self.trie.match(topic).keys())
        for ep in targets:
            ep.deliver(topic, payload, False)


class Loopback(Message):
    def __init__(self, message_handler=None, topics_subscribe=None, topic_lwt=None,
                 payload_lwt="(absent)", retain_lwt=False, bus: LoopbackBus | None = None):
        self.bus = bus or LoopbackBus()
        self.message_handler = message_handler
        self.lwt = (topic_lwt, payload_lwt, retain_lwt) if topic_lwt else None
        self.subscriptions: set = set()
        self.connected = True
        with self.bus.lock:
            self.bus.endpoints.append(self)
        if topics_subscribe:
            self.subscribe(list(topics_subscribe))

    def is_connected(self):
        return self.connected

    def deliver(self, topic, payload, retain):
        if self.connected and self.message_handler:
            self.message_handler(self, None, MQTTMessage(topic, payload, 0, retain))

    def publish(self, topic, payload, retain=False, wait=False):
        plan = _fault.active()
        if plan is not None and plan.should_drop(topic):
            return
        if isinstance(payload, str):
            payload = payload.encode("utf-8")
        self.bus.route(topic, bytes(payload or b""), retain)

    def subscribe(self, topics):
        if isinstance(topics, str):
            topics = [topics]
        for t in topics:
            with self.bus.lock:
                if t in self.subscriptions:
                    continue
                self.subscriptions.add(t)
                self.bus.trie.add(t, self)
                retained = [(rt, p) for rt, p in self.bus.retained.items() if C.topic_matches(t, rt)]
            for rt, p in retained:
                self.deliver(rt, p, True)

    def unsubscribe(self, topics):
        if isinstance(topics, str):
            topics = [topics]
        with self.bus.lock:
            for t in topics:
                if t in self.subscriptions:
                    self.subscriptions.discard(t)
                    self.bus.trie.remove(t, self)

    def set_last_will_and_testament(self, topic_lwt, payload_lwt="(absent)", retain_lwt=False):
        self.lwt = (topic_lwt, payload_lwt, retain_lwt)

    def simulate_disconnect(self):
        """Abnormal disconnect: unsubscribe everything and fire the last will."""
        self.unsubscribe(list(self.subscriptions))
        self.connected = False
        if self.lwt:
            t, p, r = self.lwt
            self.bus.route(t, p.encode() if isinstance(p, str) else p, r)

    def terminate(self):
        self.unsubscribe(list(self.subscriptions))
        self.connected = False


class MQTT(Message):
    """MQTT transport of a process: one client connection, subscriptions replayed on connect.

    Raises ``SystemError`` when no broker is reachable (like the reference), so the process
    can fall back to ``Castaway`` when ``mqtt_connection_required=False``.
    """

    def __init__(self, message_handler=None, topics_subscribe=None, topic_lwt=None,
                 payload_lwt="(absent)", retain_lwt=False):
        self.message_handler = message_handler
        self.topics_subscribe = topics_subscribe if topics_subscribe is not None else {}
        self.lwt = (topic_lwt, payload_lwt, retain_lwt) if topic_lwt else None
        self._lock = threading.RLock()
        self._subscribed: set = set()
        (server_up, self.host, self.port, self.transport, self.username, self.password,
         self.tls) = get_mqtt_configuration()
        # AIKO_MQTT_TRANSPORT: "tcp" or "websockets" (reference main/message/mqtt.py:87,108); an
        # unknown value raises here instead of silently trying plain TCP
        self.websockets = is_websocket_transport(self.transport)
        self.ws_path = os.environ.get("AIKO_MQTT_WS_PATH", "/mqtt")
        if not server_up:
            raise SystemError(f"Couldn't connect to MQTT server {self.host}:{self.port}")
        self.client = None
        self._terminating = False
        self.reconnects = 0
        self._conn_lock = threading.RLock()   # one live connection: connect / swap / reconnect serialised
        self._connect()

    def _connect(self):
        with self._conn_lock:
            self._connect_locked()

    def _connect_locked(self):
        previous = self.client
        if previous is not None and previous.is_connected():
            previous.disconnect()              # never two live connections (double delivery)
        client = MQTTClient(on_message=self._on_message, on_disconnect=self._on_disconnect)
        if self.lwt:
            client.will_set(self.lwt[0], self.lwt[1], self.lwt[2])
        try:
            client.connect(self.host, self.port, keepalive=int(os.environ.get("AIKO_MQTT_KEEPALIVE", 60)),
                           username=self.username, password=self.password, tls=self.tls,
                           transport="websockets" if self.websockets else "tcp", ws_path=self.ws_path)
        except (OSError, ConnectionError) as exc:
            raise SystemError(f"Couldn't connect to MQTT server {self.host}:{self.port}: {exc}")
        self.client = client
        with self._lock:
            topics = list(self.topics_subscribe) if not isinstance(self.topics_subscribe, str) \
                else [self.topics_subscribe]
            topics += [t for t in self._subscribed if t not in topics]   # replay after a reconnect
            self._subscribed.clear()
        if topics:
            self.subscribe(topics)

    def _on_disconnect(self, client, userdata, rc):
        """Broker lost (rc != 0): reconnect in the background with capped exponential backoff
        and replay every subscription (the reference left this as a TODO)."""
        if rc == 0 or self._terminating or client is not self.client:
            return
        threading.Thread(target=self._reconnect_loop, args=(client,), name="aiko-mqtt-reconnect",
                         daemon=True).start()

    def _reconnect_loop(self, lost):
        delay = 0.2
        while not self._terminating:
            time.sleep(delay)
            with self._conn_lock:
                if self.client is not lost:        # replaced meanwhile (will swap, another loop)
                    return
                try:
                    self._connect_locked()
                    self.reconnects += 1
                    return
                except SystemError:
                    delay = min(delay * 2, 5.0)

    def _on_message(self, client, userdata, message):
        # only the current connection delivers: a replaced one that the broker has not yet
        # dropped must not hand the process a second copy of every message
        if self.message_handler and client is self.client:
            self.message_handler(client, userdata, message)

    def is_connected(self):
        return self.client is not None and self.client.is_connected()

    def publish(self, topic, payload, retain=False, wait=False):
        plan = _fault.active()
        if plan is not None and plan.should_drop(topic):
            return
        if self.client is None:
            return
        try:
            self.client.publish(topic, payload, qos=1 if wait else 0, retain=retain, wait=wait)
        except (OSError, ConnectionError):
            pass

    def subscribe(self, topics):
        if isinstance(topics, str):
            topics = [topics]
        with self._lock:
            new = [t for t in topics if t not in self._subscribed]
            self._subscribed.update(new)
        if new and self.client is not None:
            # ordering on the single TCP connection makes SUBACK-waiting unnecessary
            self.client.subscribe([(t, 0) for t in new], wait=False)

    def unsubscribe(self, topics):
        if isinstance(topics, str):
            topics = [topics]
        with self._lock:
            gone = [t for t in topics if t in self._subscribed]
            self._subscribed.difference_update(gone)
        if gone and self.client is not None:
            self.client.unsubscribe(gone, wait=False)

    def set_last_will_and_testament(self, topic_lwt, payload_lwt="(absent)", retain_lwt=False):
        """MQTT fixes the will at CONNECT: reconnect with the new one (as the reference does)."""
        self.lwt = (topic_lwt, payload_lwt, retain_lwt)
        with self._conn_lock:
            old = self.client
            if old is not None:
                old.disconnect()
            self._connect_locked()

    def terminate(self):
        self._terminating = True
        if self.client is not None:
            self.client.disconnect()
            self.client = None
