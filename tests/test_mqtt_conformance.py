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
