"""MQTT 3.1.1 packet encoding/decoding shared by the in-repo client and broker.

The reference depends on paho-mqtt + an external mosquitto broker; neither exists on the
MI355X boxes, so the control plane carries its own implementation of the protocol subset
aiko uses: CONNECT (clean session, keep-alive, will topic/payload/retain, username/password),
CONNACK, PUBLISH (QoS 0/1, retain), PUBACK, SUBSCRIBE/SUBACK, UNSUBSCRIBE/UNSUBACK,
PINGREQ/PINGRESP, DISCONNECT.  Topic filters support ``+`` and ``#`` per the specification.
"""
from __future__ import annotations

import struct

CONNECT, CONNACK, PUBLISH, PUBACK = 1, 2, 3, 4
SUBSCRIBE, SUBACK, UNSUBSCRIBE, UNSUBACK = 8, 9, 10, 11
PINGREQ, PINGRESP, DISCONNECT = 12, 13, 14

PROTOCOL_NAME = b"MQTT"
PROTOCOL_LEVEL = 4


def encode_varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n % 128
        n //= 128
        if n:
            b |= 0x80
        out.append(b)
        if not n:
            return bytes(out)


def encode_str(s) -> bytes:
    if isinstance(s, str):
        s = s.encode("utf-8")
    return struct.pack("!H", len(s)) + s


def packet(ptype: int, flags: int, body: bytes) -> bytes:
    return bytes([(ptype << 4) | flags]) + encode_varint(len(body)) + body


def connect_packet(client_id: str, keepalive: int = 60, will_topic=None, will_payload=b"",
                   will_retain=False, will_qos=0, username=None, password=None,
                   clean_session=True) -> bytes:
    flags = 0x02 if clean_session else 0
    payload = encode_str(client_id)
    if will_topic is not None:
        flags |= 0x04 | (will_qos << 3) | (0x20 if will_retain else 0)
        if isinstance(will_payload, str):
            will_payload = will_payload.encode("utf-8")
        payload += encode_str(will_topic) + struct.pack("!H", len(will_payload)) + will_payload
    if username is not None:
        flags |= 0x80
        payload += encode_str(username)
        if password is not None:
            flags |= 0x40
            payload += encode_str(password)
    body = encode_str(PROTOCOL_NAME) + bytes([PROTOCOL_LEVEL, flags]) + struct.pack("!H", keepalive)
    return packet(CONNECT, 0, body + payload)


def publish_packet(topic: str, payload, qos: int = 0, retain: bool = False, packet_id: int = 0,
                   dup: bool = False) -> bytes:
    if isinstance(payload, str):
        payload = payload.encode("utf-8")
    elif payload is None:
        payload = b""
    body = encode_str(topic)
    if qos:
        body += struct.pack("!H", packet_id)
    flags = (0x08 if dup else 0) | (qos << 1) | (1 if retain else 0)
    return packet(PUBLISH, flags, body + bytes(payload))


def subscribe_packet(packet_id: int, topics) -> bytes:
    body = struct.pack("!H", packet_id)
    for topic, qos in topics:
        body += encode_str(topic) + bytes([qos])
    return packet(SUBSCRIBE, 0x02, body)


def unsubscribe_packet(packet_id: int, topics) -> bytes:
    body = struct.pack("!H", packet_id)
    for topic in topics:
        body += encode_str(topic)
    return packet(UNSUBSCRIBE, 0x02, body)


class PacketReader:
    """Incremental parser: feed bytes, iterate complete (type, flags, body) packets."""

    def __init__(self):
        self.buf = bytearray()

    def feed(self, data: bytes):
        self.buf += data

    def packets(self):
        buf = self.buf
        while True:
            if len(buf) < 2:
                return
            mult, length, i = 1, 0, 1
            while True:
                if i >= len(buf):
                    return
                b = buf[i]
                length += (b & 0x7F) * mult
                mult *= 128
                i += 1
                if not b & 0x80:
                    break
                if i > 4:
                    raise ValueError("malformed remaining length")
            if len(buf) < i + length:
                return
            header = buf[0]
            body = bytes(buf[i:i + length])
            del buf[:i + length]
            yield header >> 4, header & 0x0F, body


def decode_str(body: bytes, off: int):
    (n,) = struct.unpack_from("!H", body, off)
    off += 2
    return body[off:off + n].decode("utf-8"), off + n


def decode_publish(flags: int, body: bytes):
    qos = (flags >> 1) & 3
    retain = bool(flags & 1)
    topic, off = decode_str(body, 0)
    packet_id = 0
    if qos:
        (packet_id,) = struct.unpack_from("!H", body, off)
        off += 2
    return topic, body[off:], qos, retain, packet_id


def decode_connect(body: bytes) -> dict:
    name, off = decode_str(body, 0)
    level = body[off]
    flags = body[off + 1]
    (keepalive,) = struct.unpack_from("!H", body, off + 2)
    off += 4
    client_id, off = decode_str(body, off)
    info = {"protocol": name, "level": level, "keepalive": keepalive, "client_id": client_id,
            "clean_session": bool(flags & 0x02), "will": None, "username": None, "password": None}
    if flags & 0x04:
        wtopic, off = decode_str(body, off)
        (n,) = struct.unpack_from("!H", body, off)
        off += 2
        info["will"] = (wtopic, body[off:off + n], (flags >> 3) & 3, bool(flags & 0x20))
        off += n
    if flags & 0x80:
        info["username"], off = decode_str(body, off)
    if flags & 0x40:
        (n,) = struct.unpack_from("!H", body, off)
        off += 2
        info["password"] = body[off:off + n].decode("utf-8", "replace")
        off += n
    return info


def topic_matches(filter_: str, topic: str) -> bool:
    """MQTT topic filter matching (``+`` one level, ``#`` any remaining levels)."""
    if filter_ == topic:
        return True
    f = filter_.split("/")
    t = topic.split("/")
    if topic.startswith("$") and f[0] in ("+", "#"):
        return False                   # 4.7.2: wildcards at the first level never match $-topics
    for i, level in enumerate(f):
        if level == "#":
            return i == len(f) - 1
        if i >= len(t):
            return False
        if level != "+" and level != t[i]:
            return False
    return len(f) == len(t)


class TopicTrie:
    """Subscription index: filter -> set(subscriber), matched in O(topic depth)."""

    __slots__ = ("root",)

    def __init__(self):
        self.root = {"c": {}, "s": {}}

    def add(self, filter_: str, key, value=None):
        node = self.root
        for level in filter_.split("/"):
            node = node["c"].setdefault(level, {"c": {}, "s": {}})
        node["s"][key] = value
        return node

    def remove(self, filter_: str, key) -> bool:
        path = [self.root]
        node = self.root
        levels = filter_.split("/")
        for level in levels:
            node = node["c"].get(level)
            if node is None:
                return False
            path.append(node)
        if key not in node["s"]:
            return False
        del node["s"][key]
        for level, (parent, child) in zip(reversed(levels), zip(reversed(path[:-1]), reversed(path[1:]))):
            if child["s"] or child["c"]:
                break
            del parent["c"][level]
        return True

    def match(self, topic: str) -> dict:
        """Return {key: value} of every subscription matching ``topic``."""
        out: dict = {}
        levels = topic.split("/")
        n = len(levels)
        stack = [(self.root, 0)]
        while stack:
            node, i = stack.pop()
            children = node["c"]
            h = children.get("#")
            if h is not None and not (i == 0 and levels[0].startswith("$")):
                out.update(h["s"])
            if i == n:
                out.update(node["s"])
                continue
            c = children.get(levels[i])
            if c is not None:
                stack.append((c, i + 1))
            p = children.get("+")
            if p is not None and not (i == 0 and levels[0].startswith("$")):
                stack.append((p, i + 1))
        return out
