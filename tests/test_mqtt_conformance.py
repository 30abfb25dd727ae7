"""MQTT 3.1.1 conformance vectors (OASIS mqtt-v3.1.1-os), byte-exact.

mosquitto / paho cannot be installed here, so interoperability is pinned to the
specification's own non-normative examples instead: remaining-length encoding (table 2.4),
UTF-8 string encoding (1.5.3), the CONNECT variable header example (3.1.2.10, flags 0xCE),
PUBLISH / SUBSCRIBE / UNSUBSCRIBE variable-header and payload examples (3.3.2.3, 3.8.3.2,
3.10.3.2), the fixed two-byte PINGREQ / PINGRESP / DISCONNECT packets, and the topic-filter
wildcard rules (4.7.1, 4.7.2 incl. ``$``-topics)."""
import pytest

from aiko_services_amd.message import mqtt_codec as C


@pytest.mark.parametrize("n,enc", [
    (0, b"\x00"), (127, b"\x7f"), (128, b"\x80\x01"), (16383, b"\xff\x7f"), (16384, b"\x80\x80\x01"),
    (2097151, b"\xff\xff\x7f"), (2097152, b"\x80\x80\x80\x01"), (268435455, b"\xff\xff\xff\x7f")])
def test_remaining_length_table_2_4(n, enc):
    assert C.encode_varint(n) == enc
    r = C.PacketReader()
    r.feed(bytes([0x30]) + enc + b"\x00" * n if n < 20000 else b"")
    if n < 20000:
        (ptype, flags, body), = list(r.packets())
        assert ptype == C.PUBLISH and len(body) == n


def test_utf8_string_1_5_3():
    assert C.encode_str("A\U0002A6D4") == b"\x00\x05\x41\xf0\xaa\x9b\x94"
    assert C.decode_str(b"\x00\x05\x41\xf0\xaa\x9b\x94", 0)[0] == "A\U0002A6D4"


def test_connect_3_1_2_10_flags_and_header():
    pkt = C.connect_packet("cid", keepalive=10, will_topic="w", will_payload=b"bye", will_qos=1,
                           username="u", password="p", clean_session=True)
    assert pkt[0] == 0x10
    body = pkt[2:]
    assert body[:10] == b"\x00\x04MQTT\x04\xce\x00\x0a"      # protocol name, level 4, 0xCE, keep alive 10
    assert body[10:] == b"\x00\x03cid" + b"\x00\x01w" + b"\x00\x03bye" + b"\x00\x01u" + b"\x00\x01p"
    assert pkt[1] == len(body)
    d = C.decode_connect(body)
    assert d["client_id"] == "cid" and d["keepalive"] == 10 and d["clean_session"]
    assert d["will"] == ("w", b"bye", 1, False) and d["username"] == "u" and d["password"] == "p"


def test_connect_minimal_clean_session():
    assert C.connect_packet("", keepalive=60) == b"\x10\x0c\x00\x04MQTT\x04\x02\x00\x3c\x00\x00"


def test_publish_3_3_2_3_and_retain_qos_flags():
    pkt = C.publish_packet("a/b", b"", qos=1, packet_id=10)
    assert pkt == b"\x32\x07\x00\x03a/b\x00\x0a"
    assert C.publish_packet("a/b", b"hi", qos=0, retain=True) == b"\x31\x07\x00\x03a/bhi"
    assert C.publish_packet("a/b", b"", qos=1, packet_id=10, dup=True)[0] == 0x3a
    assert C.decode_publish(pkt[0] & 0x0F, pkt[2:]) == ("a/b", b"", 1, False, 10)


def test_subscribe_3_8_3_2():
    assert C.subscribe_packet(10, [("a/b", 1), ("c/d", 2)]) == \
        b"\x82\x0e\x00\x0a\x00\x03a/b\x01\x00\x03c/d\x02"


def test_unsubscribe_3_10_3_2():
    assert C.unsubscribe_packet(10, ["a/b", "c/d"]) == b"\xa2\x0c\x00\x0a\x00\x03a/b\x00\x03c/d"


def test_fixed_two_byte_packets():
    assert C.packet(C.PINGREQ, 0, b"") == b"\xc0\x00"
    assert C.packet(C.PINGRESP, 0, b"") == b"\xd0\x00"
    assert C.packet(C.DISCONNECT, 0, b"") == b"\xe0\x00"


@pytest.mark.parametrize("filt,topic,match", [
    ("sport/tennis/player1/#", "sport/tennis/player1", True),
    ("sport/tennis/player1/#", "sport/tennis/player1/ranking", True),
    ("sport/tennis/player1/#", "sport/tennis/player1/score/wimbledon", True),
    ("sport/#", "sport", True),
    ("#", "sport/tennis", True),
    ("sport/tennis/+", "sport/tennis/player1", True),
    ("sport/tennis/+", "sport/tennis/player1/ranking", False),
    ("sport/+", "sport", False),
    ("sport/+", "sport/", True),
    ("+/+", "/finance", True),
    ("/+", "/finance", True),
    ("+", "/finance", False),
    ("#", "$SYS/broker/clients", False),
    ("+/monitor/Clients", "$SYS/monitor/Clients", False),
    ("$SYS/#", "$SYS/broker/clients", True),
    ("$SYS/monitor/+", "$SYS/monitor/Clients", True),
])
def test_topic_filters_4_7(filt, topic, match):
    assert C.topic_matches(filt, topic) is match
    trie = C.TopicTrie()
    trie.add(filt, "sub", 0)
    assert (len(trie.match(topic)) > 0) is match


# ---- MQTT over WebSockets (RFC 6455): byte-exact handshake and frame vectors -------------------
from aiko_services_amd.message import websocket as WS  # noqa: E402


def test_ws_accept_key_rfc6455_1_3():
    # the worked example of RFC 6455 section 1.3
    assert WS.accept_key("dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_ws_handshake_bytes():
    req = WS.client_request("broker", 9001, "/mqtt", "dGhlIHNhbXBsZSBub25jZQ==")
    assert req == (b"GET /mqtt HTTP/1.1\r\nHost: broker:9001\r\nUpgrade: websocket\r\n"
                   b"Connection: Upgrade\r\nSec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\n"
                   b"Sec-WebSocket-Version: 13\r\nSec-WebSocket-Protocol: mqtt\r\n\r\n")
    assert WS.server_response("dGhlIHNhbXBsZSBub25jZQ==") == (
        b"HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
        b"Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\nSec-WebSocket-Protocol: mqtt\r\n\r\n")
    # the broker side answers a client request with exactly that response
    s = WS.ServerSession()
    app, reply, close = s.feed(req)
    assert (app, close) == (b"", False) and reply == WS.server_response("dGhlIHNhbXBsZSBub25jZQ==")


KEY = bytes([0x37, 0xFA, 0x21, 0x3D])


def test_ws_frames_rfc6455_5_7():
    # single-frame unmasked text "Hello"
    assert WS.encode_frame(b"Hello", WS.OP_TEXT) == bytes([0x81, 0x05, 0x48, 0x65, 0x6C, 0x6C, 0x6F])
    # single-frame masked text "Hello"
    masked = bytes([0x81, 0x85, 0x37, 0xFA, 0x21, 0x3D, 0x7F, 0x9F, 0x4D, 0x51, 0x58])
    assert WS.encode_frame(b"Hello", WS.OP_TEXT, KEY) == masked
    assert WS.FrameDecoder(require_mask=True).feed(masked) == [(WS.OP_TEXT, b"Hello")]
    # fragmented unmasked text: "Hel" + "lo"
    frag = bytes([0x01, 0x03, 0x48, 0x65, 0x6C, 0x80, 0x02, 0x6C, 0x6F])
    assert WS.encode_frame(b"Hel", WS.OP_TEXT, fin=False) + WS.encode_frame(b"lo", WS.OP_CONT) == frag
    assert WS.FrameDecoder(require_mask=False).feed(frag) == [(WS.OP_TEXT, b"Hello")]
    # unmasked ping / masked pong
    assert WS.encode_frame(b"Hello", WS.OP_PING) == bytes([0x89, 0x05]) + b"Hello"
    assert WS.encode_frame(b"Hello", WS.OP_PONG, KEY) == bytes([0x8A, 0x85, 0x37, 0xFA, 0x21, 0x3D,
                                                                 0x7F, 0x9F, 0x4D, 0x51, 0x58])
    # 256 bytes (16-bit length) and 64 KiB (64-bit length) unmasked binary
    assert WS.encode_frame(bytes(256))[:4] == bytes([0x82, 0x7E, 0x01, 0x00])
    assert WS.encode_frame(bytes(65536))[:10] == bytes([0x82, 0x7F, 0, 0, 0, 0, 0, 1, 0, 0])


def test_ws_decoder_incremental_and_rules():
    import pytest as _pytest
    blob = bytes(range(256)) * 300
    frame = WS.encode_frame(blob, WS.OP_BINARY, KEY)
    d = WS.FrameDecoder(require_mask=True)
    got = []
    for i in range(0, len(frame), 7):                     # byte-dribbled
        got += d.feed(frame[i:i + 7])
    assert got == [(WS.OP_BINARY, blob)]
    with _pytest.raises(ValueError):                      # client frames must be masked
        WS.FrameDecoder(require_mask=True).feed(WS.encode_frame(b"x"))
    with _pytest.raises(ValueError):                      # server frames must not be
        WS.FrameDecoder(require_mask=False).feed(WS.encode_frame(b"x", WS.OP_BINARY, KEY))


def test_ws_transport_names():
    import pytest as _pytest
    assert WS.is_websocket_transport("websockets") and not WS.is_websocket_transport("tcp")
    with _pytest.raises(ValueError):
        WS.is_websocket_transport("carrier-pigeon")
