"""Minimal MQTT 3.1.1 client (replaces paho-mqtt, which is not installed on the boxes).

A dedicated network thread reads the socket and invokes ``on_message(client, userdata,
message)`` with a paho-compatible ``message`` (``.topic`` str, ``.payload`` bytes,
``.retain``, ``.qos``).  ``publish`` writes directly from the caller's thread under a lock
(TCP_NODELAY, no busy-wait), ``connect`` waits on a condition for CONNACK instead of the
reference's 2000 x 1 ms polling loop (``message/mqtt.py:255-289``).  Keep-alive PINGREQs are
sent by the network thread.  TLS is supported via ``ssl`` when requested, and MQTT over
WebSockets (``transport="websockets"``, ``message/websocket.py``) like paho's transport option.
"""
from __future__ import annotations

import itertools
import socket
import ssl
import struct
import threading
import time
import uuid
from dataclasses import dataclass

from . import mqtt_codec as C
from .websocket import client_connect, is_websocket_transport

__all__ = ["MQTTClient", "MQTTMessage"]


@dataclass
class MQTTMessage:
    topic: str
    payload: bytes
    qos: int = 0
    retain: bool = False


class MQTTClient:
    def __init__(self, client_id: str | None = None, on_message=None, on_connect=None,
                 on_disconnect=None, userdata=None):
        self.client_id = client_id or f"aiko-{uuid.uuid4().hex[:12]}"
        self.on_message = on_message
        self.on_connect = on_connect
        self.on_disconnect = on_disconnect
        self.userdata = userdata
        self.sock: socket.socket | None = None
        self._wlock = threading.Lock()
        self._cv = threading.Condition()
        self._connected = False
        self._acks: dict = {}
        self._pid = itertools.count(1)
        self._thread: threading.Thread | None = None
        self._stop = False
        self.keepalive = 60
        self._last_tx = time.monotonic()
        self.will = None
        self.host = None
        self.port = None

    # ---- connection ---------------------------------------------------------------------------
    def will_set(self, topic, payload="", retain=False, qos=0):
        self.will = (topic, payload, retain, qos)

    def connect(self, host="127.0.0.1", port=1883, keepalive=60, username=None, password=None,
                tls=False, timeout=5.0, transport="tcp", ws_path="/mqtt"):
        """``transport``: ``tcp`` or ``websockets`` (RFC 6455 Upgrade on ``ws_path``,
        subprotocol ``mqtt``; over TLS when ``tls``); any other value raises ``ValueError``."""
        websockets = is_websocket_transport(transport)
        self.host, self.port, self.keepalive = host, port, keepalive
        sock = socket.create_connection((host, port), timeout=timeout)
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if tls:
            ctx = ssl.create_default_context()
            sock = ctx.wrap_socket(sock, server_hostname=host)
        if websockets:
            try:
                sock = client_connect(sock, host, port, ws_path)
            except (OSError, ConnectionError):
                sock.close()
                raise
        sock.settimeout(None)
        self.sock = sock
        self._stop = False
        w = self.will
        pkt = C.connect_packet(self.client_id, keepalive,
                               will_topic=w[0] if w else None, will_payload=w[1] if w else b"",
                               will_retain=w[2] if w else False, will_qos=w[3] if w else 0,
                               username=username, password=password)
        self._thread = threading.Thread(target=self._reader, name="aiko-mqtt-net", daemon=True)
        self._thread.start()
        self._write(pkt)
        with self._cv:
            if not self._cv.wait_for(lambda: self._connected or self._stop, timeout):
                raise ConnectionError(f"MQTT CONNACK timeout from {host}:{port}")
            if not self._connected:
                raise ConnectionError(f"MQTT connection refused by {host}:{port}")
        return 0

    def is_connected(self):
        return self._connected

    def disconnect(self):
        if self.sock is None:
            return
        try:
            self._write(C.packet(C.DISCONNECT, 0, b""))
        except OSError:
            pass
        self._shutdown()

    def _shutdown(self):
        self._stop = True
        sock, self.sock = self.sock, None
        if sock is not None:
            try:
                sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass
            try:
                sock.close()
            except OSError:
                pass
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(timeout=2.0)
        with self._cv:
            was = self._connected
            self._connected = False
            self._cv.notify_all()
        if was and self.on_disconnect:
            self.on_disconnect(self, self.userdata, 0)

    # ---- I/O ---------------------------------------------------------------------------------
    def _write(self, data: bytes):
        sock = self.sock
        if sock is None:
            raise ConnectionError("MQTT client not connected")
        with self._wlock:
            sock.sendall(data)
            self._last_tx = time.monotonic()

    def _reader(self):
        reader = C.PacketReader()
        sock = self.sock
        sock_timeout = max(1.0, self.keepalive / 2) if self.keepalive else None
        sock.settimeout(sock_timeout)
        try:
            while not self._stop:
                try:
                    data = sock.recv(65536)
                except socket.timeout:
                    if self.keepalive and time.monotonic() - self._last_tx > self.keepalive / 2:
                        self._write(C.packet(C.PINGREQ, 0, b""))
                    continue
                if not data:
                    break
                reader.feed(data)
                for ptype, flags, body in reader.packets():
                    self._dispatch(ptype, flags, body)
                if self.keepalive and time.monotonic() - self._last_tx > self.keepalive / 2:
                    self._write(C.packet(C.PINGREQ, 0, b""))
        except (OSError, ValueError):
            pass
        finally:
            if not self._stop:
                self._stop = True
                with self._cv:
                    was = self._connected
                    self._connected = False
                    self._cv.notify_all()
                if was and self.on_disconnect:
                    self.on_disconnect(self, self.userdata, 1)

    def _dispatch(self, ptype, flags, body):
        if ptype == C.CONNACK:
            ok = len(body) >= 2 and body[1] == 0
            with self._cv:
                self._connected = ok
                if not ok:
                    self._stop = True
                self._cv.notify_all()
            if ok and self.on_connect:
                self.on_connect(self, self.userdata, {}, 0)
        elif ptype == C.PUBLISH:
            topic, payload, qos, retain, pid = C.decode_publish(flags, body)
            if qos == 1:
                self._write(C.packet(C.PUBACK, 0, struct.pack("!H", pid)))
            if self.on_message:
                self.on_message(self, self.userdata, MQTTMessage(topic, payload, qos, retain))
        elif ptype in (C.SUBACK, C.UNSUBACK, C.PUBACK):
            (pid,) = struct.unpack_from("!H", body, 0)
            with self._cv:
                self._acks[pid] = True
                self._cv.notify_all()

    def _next_pid(self):
        pid = next(self._pid) & 0xFFFF
        return pid or next(self._pid) & 0xFFFF

    def _wait_ack(self, pid, timeout):
        with self._cv:
            ok = self._cv.wait_for(lambda: self._acks.pop(pid, None) is not None or not self._connected,
                                   timeout)
        return ok

    # ---- API ---------------------------------------------------------------------------------
    def publish(self, topic, payload=b"", qos=0, retain=False, wait=False, timeout=5.0):
        pid = self._next_pid() if qos else 0
        self._write(C.publish_packet(topic, payload, qos, retain, pid))
        if qos and wait:
            return self._wait_ack(pid, timeout)
        return True

    def subscribe(self, topics, qos=0, wait=True, timeout=5.0):
        if isinstance(topics, str):
            topics = [(topics, qos)]
        topics = [(t, q) if isinstance(t, str) else t for t, q in
                  [(x, qos) if isinstance(x, str) else x for x in topics]]
        if not topics:
            return True
        pid = self._next_pid()
        self._write(C.subscribe_packet(pid, topics))
        return self._wait_ack(pid, timeout) if wait else True

    def unsubscribe(self, topics, wait=True, timeout=5.0):
        if isinstance(topics, str):
            topics = [topics]
        pid = self._next_pid()
        self._write(C.unsubscribe_packet(pid, topics))
        return self._wait_ack(pid, timeout) if wait else True
