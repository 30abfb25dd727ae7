"""MQTT over WebSockets (RFC 6455, subprotocol ``mqtt``) for the in-repo client and broker.

The reference hands ``AIKO_MQTT_TRANSPORT`` to paho (``mqtt.Client(transport=...)``,
``/root/reference/src/aiko_services/main/message/mqtt.py:87,108``), so a deployment behind a
WebSocket-only proxy sets ``AIKO_MQTT_TRANSPORT=websockets``.  Here:

* :func:`client_connect` performs the HTTP/1.1 Upgrade handshake on a connected (optionally TLS)
  socket and returns a :class:`WebSocketStream`: a socket-like object (``sendall`` / ``recv`` /
  ``settimeout`` / ``shutdown`` / ``close``) the MQTT client uses unchanged — every MQTT write is
  one masked binary frame, ``recv`` returns the payload bytes of the next data frames (ping ->
  pong answered inline, close -> ``b""``);
* :class:`ServerSession` is the broker side, driven by its non-blocking selector loop: ``feed``
  takes raw socket bytes and returns (MQTT bytes, bytes to send back, closed); ``wrap`` frames
  broker output (unmasked binary frames).

Frames: FIN + opcode, 7 / 16 / 64-bit lengths, 4-byte masking key (client -> server frames MUST
be masked, server -> client MUST NOT: the server closes a connection that sends unmasked data),
continuation frames reassembled, control frames (ping / pong / close) interleaved.
"""
from __future__ import annotations

import base64
import hashlib
import os
import struct
import threading

__all__ = ["GUID", "accept_key", "encode_frame", "FrameDecoder", "WebSocketStream", "client_connect",
           "ServerSession", "OP_CONT", "OP_TEXT", "OP_BINARY", "OP_CLOSE", "OP_PING", "OP_PONG"]

GUID = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
OP_CONT, OP_TEXT, OP_BINARY, OP_CLOSE, OP_PING, OP_PONG = 0x0, 0x1, 0x2, 0x8, 0x9, 0xA
_MAX_HEADER = 16384
_MAX_MESSAGE = 256 << 20


def accept_key(key: str) -> str:
    """``Sec-WebSocket-Accept`` for a ``Sec-WebSocket-Key`` (RFC 6455 §4.2.2)."""
    return base64.b64encode(hashlib.sha1((key + GUID).encode("ascii")).digest()).decode("ascii")


def _mask(data: bytes, key: bytes) -> bytes:
    n = len(data)
    if n == 0:
        return b""
    k = (key * (n // 4 + 1))[:n]
    return (int.from_bytes(data, "little") ^ int.from_bytes(k, "little")).to_bytes(n, "little")


def encode_frame(payload: bytes, opcode: int = OP_BINARY, mask_key: bytes | None = None, fin: bool = True) -> bytes:
    """One frame; ``mask_key`` (4 bytes) masks it (client -> server)."""
    payload = bytes(payload)
    n = len(payload)
    head = bytearray([(0x80 if fin else 0) | opcode])
    m = 0x80 if mask_key is not None else 0
    if n < 126:
        head.append(m | n)
    elif n < 1 << 16:
        head.append(m | 126)
        head += struct.pack("!H", n)
    else:
        head.append(m | 127)
        head += struct.pack("!Q", n)
    if mask_key is not None:
        if len(mask_key) != 4:
            raise ValueError("masking key must be 4 bytes")
        return bytes(head) + mask_key + _mask(payload, mask_key)
    return bytes(head) + payload


class FrameDecoder:
    """Incremental frame parser: ``feed(data)`` -> list of complete messages ``(opcode, payload)``
    (data messages reassembled from continuations; control frames returned as they come).
    ``require_mask``: True on the server (client frames must be masked), False on the client
    (server frames must not be)."""

    def __init__(self, require_mask: bool):
        self.require_mask = require_mask
        self.buf = bytearray()
        self._frag_op = None
        self._frag = bytearray()

    def feed(self, data: bytes) -> list:
        self.buf += data
        out = []
        while True:
            b = self.buf
            if len(b) < 2:
                break
            fin, op = b[0] & 0x80, b[0] & 0x0F
            if b[0] & 0x70:
                raise ValueError("websocket: reserved bits set (no extension negotiated)")
            masked, n = b[1] & 0x80, b[1] & 0x7F
            off = 2
            if n == 126:
                if len(b) < 4:
                    break
                (n,) = struct.unpack_from("!H", b, 2)
                off = 4
            elif n == 127:
                if len(b) < 10:
                    break
                (n,) = struct.unpack_from("!Q", b, 2)
                off = 10
            if n > _MAX_MESSAGE:
                raise ValueError("websocket: frame too large")
            if bool(masked) != self.require_mask:
                raise ValueError("websocket: masking violates RFC 6455 5.1")
            key = b""
            if masked:
                if len(b) < off + 4:
                    break
                key = bytes(b[off:off + 4])
                off += 4
            if len(b) < off + n:
                break
            payload = bytes(b[off:off + n])
            del b[:off + n]
            if masked:
                payload = _mask(payload, key)
            if op >= 0x8:                                   # control frame
                if not fin or n > 125:
                    raise ValueError("websocket: fragmented or oversized control frame")
                out.append((op, payload))
            elif op == OP_CONT:
                if self._frag_op is None:
                    raise ValueError("websocket: continuation without a first frame")
                self._frag += payload
                if len(self._frag) > _MAX_MESSAGE:
                    raise ValueError("websocket: message too large")
                if fin:
                    out.append((self._frag_op, bytes(self._frag)))
                    self._frag_op, self._frag = None, bytearray()
            elif op in (OP_TEXT, OP_BINARY):
                if self._frag_op is not None:
                    raise ValueError("websocket: new message inside a fragmented one")
                if fin:
                    out.append((op, payload))
                else:
                    self._frag_op, self._frag = op, bytearray(payload)
            else:
                raise ValueError(f"websocket: unknown opcode {op}")
        return out


def _read_http_head(sock, leftover: bytes = b"") -> tuple[bytes, bytes]:
    buf = bytearray(leftover)
    while b"\r\n\r\n" not in buf:
        if len(buf) > _MAX_HEADER:
            raise ConnectionError("websocket: HTTP header too large")
        chunk = sock.recv(4096)
        if not chunk:
            raise ConnectionError("websocket: connection closed during the handshake")
        buf += chunk
    i = buf.index(b"\r\n\r\n") + 4
    return bytes(buf[:i]), bytes(buf[i:])


def _headers(head: bytes) -> tuple[str, dict]:
    lines = head.decode("iso-8859-1").split("\r\n")
    fields = {}
    for line in lines[1:]:
        if ":" in line:
            k, v = line.split(":", 1)
            fields[k.strip().lower()] = v.strip()
    return lines[0], fields


def client_request(host: str, port: int, path: str, key: str, subprotocol: str = "mqtt") -> bytes:
    """The client's Upgrade request (byte-exact: tests/test_mqtt_conformance.py)."""
    return (f"GET {path} HTTP/1.1\r\n"
            f"Host: {host}:{port}\r\n"
            "Upgrade: websocket\r\n"
            "Connection: Upgrade\r\n"
            f"Sec-WebSocket-Key: {key}\r\n"
            "Sec-WebSocket-Version: 13\r\n"
            f"Sec-WebSocket-Protocol: {subprotocol}\r\n"
            "\r\n").encode("ascii")


def server_response(key: str, subprotocol: str | None = "mqtt") -> bytes:
    """The server's 101 response (byte-exact: tests/test_mqtt_conformance.py)."""
    proto = f"Sec-WebSocket-Protocol: {subprotocol}\r\n" if subprotocol else ""
    return ("HTTP/1.1 101 Switching Protocols\r\n"
            "Upgrade: websocket\r\n"
            "Connection: Upgrade\r\n"
            f"Sec-WebSocket-Accept: {accept_key(key)}\r\n"
            f"{proto}\r\n").encode("ascii")


class WebSocketStream:
    """Client side of an established WebSocket, shaped like the socket the MQTT client uses."""

    def __init__(self, sock, leftover: bytes = b""):
        self.sock = sock
        self.decoder = FrameDecoder(require_mask=False)
        self._pending = bytearray()
        self._closed = False
        self._early = leftover
        self._lock = threading.Lock()     # frames of the writer and of inline pongs never interleave

    def _send_frame(self, payload: bytes, opcode: int):
        frame = encode_frame(payload, opcode, os.urandom(4))
        with self._lock:
            self.sock.sendall(frame)

    # socket-like API ---------------------------------------------------------------------------
    def sendall(self, data: bytes):
        self._send_frame(data, OP_BINARY)

    def recv(self, n: int) -> bytes:
        while not self._pending:
            if self._closed:
                return b""
            if self._early:
                data, self._early = self._early, b""
            else:
                data = self.sock.recv(65536)          # socket.timeout propagates (keep-alive)
            if not data:
                self._closed = True
                return b""
            for op, payload in self.decoder.feed(data):
                if op in (OP_BINARY, OP_TEXT):
                    self._pending += payload
                elif op == OP_PING:
                    self._send_frame(payload, OP_PONG)
                elif op == OP_CLOSE:
                    try:
                        self._send_frame(payload[:2], OP_CLOSE)
                    except OSError:
                        pass
                    self._closed = True
                    break
        out = bytes(self._pending[:n])
        del self._pending[:n]
        return out

    def settimeout(self, t):
        self.sock.settimeout(t)

    def setsockopt(self, *args):
        self.sock.setsockopt(*args)

    def shutdown(self, how):
        try:
            self._send_frame(struct.pack("!H", 1000), OP_CLOSE)
        except OSError:
            pass
        self.sock.shutdown(how)

    def close(self):
        self.sock.close()

    def fileno(self):
        return self.sock.fileno()


def client_connect(sock, host: str, port: int, path: str = "/mqtt", subprotocol: str = "mqtt",
                   key: str | None = None) -> WebSocketStream:
    """Upgrade a connected socket to a WebSocket (blocking handshake)."""
    key = key or base64.b64encode(os.urandom(16)).decode("ascii")
    sock.sendall(client_request(host, port, path, key, subprotocol))
    head, rest = _read_http_head(sock)
    status, fields = _headers(head)
    if not status.startswith("HTTP/1.1 101"):
        raise ConnectionError(f"websocket upgrade refused: {status}")
    if fields.get("upgrade", "").lower() != "websocket" or "upgrade" not in fields.get("connection", "").lower():
        raise ConnectionError("websocket upgrade: missing Upgrade / Connection headers")
    if fields.get("sec-websocket-accept") != accept_key(key):
        raise ConnectionError("websocket upgrade: bad Sec-WebSocket-Accept")
    proto = fields.get("sec-websocket-protocol")
    if proto is not None and proto != subprotocol:
        raise ConnectionError(f"websocket upgrade: server chose subprotocol {proto!r}")
    return WebSocketStream(sock, rest)


class ServerSession:
    """Broker side of one WebSocket connection (non-blocking: the broker loop feeds bytes)."""

    def __init__(self):
        self.open = False
        self.closed = False
        self._head = bytearray()
        self.decoder = FrameDecoder(require_mask=True)

    def feed(self, data: bytes) -> tuple[bytes, bytes, bool]:
        """-> (MQTT bytes for the packet reader, bytes to send on the socket, close now)."""
        reply = bytearray()
        if not self.open:
            self._head += data
            if b"\r\n\r\n" not in self._head:
                if len(self._head) > _MAX_HEADER:
                    return b"", b"HTTP/1.1 431 Request Header Fields Too Large\r\n\r\n", True
                return b"", b"", False
            i = self._head.index(b"\r\n\r\n") + 4
            head, data = bytes(self._head[:i]), bytes(self._head[i:])
            self._head = bytearray()
            request, fields = _headers(head)
            key = fields.get("sec-websocket-key")
            if (not request.startswith("GET ") or fields.get("upgrade", "").lower() != "websocket"
                    or key is None or fields.get("sec-websocket-version") != "13"):
                return b"", b"HTTP/1.1 400 Bad Request\r\nSec-WebSocket-Version: 13\r\n\r\n", True
            offered = [p.strip() for p in fields.get("sec-websocket-protocol", "").split(",") if p.strip()]
            if offered and "mqtt" not in offered:
                return b"", b"HTTP/1.1 400 Bad Request\r\n\r\n", True
            reply += server_response(key, "mqtt" if offered else None)
            self.open = True
            if not data:
                return b"", bytes(reply), False
        app = bytearray()
        try:
            for op, payload in self.decoder.feed(data):
                if op in (OP_BINARY, OP_TEXT):
                    app += payload
                elif op == OP_PING:
                    reply += encode_frame(payload, OP_PONG)
                elif op == OP_CLOSE:
                    reply += encode_frame(payload[:2], OP_CLOSE)
                    self.closed = True
                    return bytes(app), bytes(reply), True
        except ValueError:
            reply += encode_frame(struct.pack("!H", 1002), OP_CLOSE)      # protocol error
            return bytes(app), bytes(reply), True
        return bytes(app), bytes(reply), False

    def wrap(self, data: bytes) -> bytes:
        return encode_frame(data, OP_BINARY)


def is_websocket_transport(transport: str) -> bool:
    """``AIKO_MQTT_TRANSPORT``: ``tcp`` or ``websockets`` (paho's names); anything else raises."""
    t = (transport or "tcp").strip().lower()
    if t in ("tcp", ""):
        return False
    if t in ("websockets", "websocket", "ws"):
        return True
    raise ValueError(f"AIKO_MQTT_TRANSPORT={transport!r}: expected 'tcp' or 'websockets'")
