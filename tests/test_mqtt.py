"""In-repo MQTT 3.1.1 broker + client: pub/sub, wildcards, retained, LWT, QoS 1, topic trie."""
import queue
import socket
import threading
import time

import pytest

from aiko_services_amd.message import mqtt_codec as C
from aiko_services_amd.message.mqtt_broker import Broker, start_broker_thread
from aiko_services_amd.message.mqtt_client import MQTTClient


@pytest.fixture
def broker():
    b, port = start_broker_thread("127.0.0.1", 0)
    yield b, port
    b.stop()


def _client(port, **kw):
    q = queue.Queue()
    c = MQTTClient(on_message=lambda cl, ud, m: q.put((m.topic, m.payload, m.retain)), **kw)
    return c, q


def test_topic_matching():
    assert C.topic_matches("a/+/c", "a/b/c")
    assert not C.topic_matches("a/+/c", "a/b/d")
    assert C.topic_matches("a/#", "a/b/c/d") and C.topic_matches("a/#", "a")
    assert not C.topic_matches("a/+", "a/b/c")
    assert C.topic_matches("ns/+/+/+/state", "ns/host/12/0/state")
    t = C.TopicTrie()
    t.add("a/+/c", "k1")
    t.add("a/#", "k2")
    t.add("a/b/c", "k3")
    t.add("x/y", "k4")
    assert set(t.match("a/b/c")) == {"k1", "k2", "k3"}
    assert set(t.match("a")) == {"k2"}
    assert t.remove("a/#", "k2") and not t.remove("a/#", "k2")
    assert set(t.match("a/b/c")) == {"k1", "k3"}


def test_packet_codec_roundtrip():
    r = C.PacketReader()
    data = C.publish_packet("t/1", b"x" * 300, qos=1, retain=True, packet_id=7)
    r.feed(data[:5])
    assert list(r.packets()) == []
    r.feed(data[5:])
    (ptype, flags, body), = list(r.packets())
    assert ptype == C.PUBLISH
    assert C.decode_publish(flags, body) == ("t/1", b"x" * 300, 1, True, 7)
    info = C.decode_connect(C.connect_packet("cid", 30, "w/t", b"bye", True, 0, "u", "p")[2:])
    assert info["client_id"] == "cid" and info["will"] == ("w/t", b"bye", 0, True)
    assert info["username"] == "u" and info["password"] == "p" and info["keepalive"] == 30


def test_pubsub_wildcards_retained_qos1(broker):
    _, port = broker
    sub, q = _client(port)
    sub.connect("127.0.0.1", port)
    pub, _ = _client(port)
    pub.connect("127.0.0.1", port)
    pub.publish("ns/service/registrar", "(primary found a/b/1/1 2 0)", retain=True)
    assert sub.subscribe([("ns/+/x", 0), ("ns/service/#", 0)], wait=True)
    topic, payload, retain = q.get(timeout=2)
    assert topic == "ns/service/registrar" and retain
    pub.publish("ns/a/x", "hello")
    pub.publish("ns/a/y", "nope")
    assert pub.publish("ns/b/x", b"qos1", qos=1, wait=True)
    got = [q.get(timeout=2)[:2] for _ in range(2)]
    assert got == [("ns/a/x", b"hello"), ("ns/b/x", b"qos1")]
    assert q.empty()
    # clear the retained message
    pub.publish("ns/service/registrar", "", retain=True)
    late, lq = _client(port)
    late.connect("127.0.0.1", port)
    late.subscribe("ns/service/#", wait=True)
    time.sleep(0.2)
    assert lq.empty()
    for c in (sub, pub, late):
        c.disconnect()


def test_last_will_on_abnormal_disconnect(broker):
    _, port = broker
    watcher, q = _client(port)
    watcher.connect("127.0.0.1", port)
    watcher.subscribe("aiko/+/+/0/state", wait=True)
    victim, _ = _client(port)
    victim.will_set("aiko/h/123/0/state", "(absent)")
    victim.connect("127.0.0.1", port)
    # graceful disconnect: no will
    polite, _ = _client(port)
    polite.will_set("aiko/h/124/0/state", "(absent)")
    polite.connect("127.0.0.1", port)
    polite.disconnect()
    # abnormal: kill the socket
    victim.sock.shutdown(socket.SHUT_RDWR)
    victim.sock.close()
    topic, payload, _ = q.get(timeout=3)
    assert topic == "aiko/h/123/0/state" and payload == b"(absent)"
    time.sleep(0.2)
    assert q.empty()
    watcher.disconnect()


def test_broker_throughput(broker):
    """Control-plane message rate through the broker (reference: ~100 msgs/s per process)."""
    _, port = broker
    sub, q = _client(port)
    sub.connect("127.0.0.1", port)
    sub.subscribe("bench/#", wait=True)
    pub, _ = _client(port)
    pub.connect("127.0.0.1", port)
    n = 5000
    t0 = time.perf_counter()
    for i in range(n):
        pub.publish("bench/x", "(process_frame (stream_id: 1 frame_id: %d) (a: 0))" % i)
    for _ in range(n):
        q.get(timeout=10)
    rate = n / (time.perf_counter() - t0)
    assert rate > 2000, rate
    sub.disconnect()
    pub.disconnect()


def test_transport_reconnects_after_broker_loss(monkeypatch):
    """Broker restart: the process transport reconnects with backoff and replays subscriptions
    (the reference's MQTT class leaves reconnection as a TODO)."""
    from aiko_services_amd.message.message import MQTT

    b1, port = start_broker_thread("127.0.0.1", 0)
    monkeypatch.setenv("AIKO_MQTT_HOST", "127.0.0.1")
    monkeypatch.setenv("AIKO_MQTT_PORT", str(port))
    got = queue.Queue()
    t = MQTT(message_handler=lambda cl, ud, m: got.put(m.payload), topics_subscribe=["a/b"])
    t.subscribe(["late/#"])
    try:
        b1.stop()
        deadline = time.time() + 5
        while t.is_connected() and time.time() < deadline:
            time.sleep(0.05)
        assert not t.is_connected()
        b2 = Broker("127.0.0.1", port)
        b2.bind()
        threading.Thread(target=b2.serve_forever, daemon=True).start()
        try:
            deadline = time.time() + 10
            while not t.is_connected() and time.time() < deadline:
                time.sleep(0.05)
            assert t.is_connected() and t.reconnects == 1
            time.sleep(0.2)
            pub, _ = _client(port)
            pub.connect("127.0.0.1", port)
            pub.publish("a/b", b"one")
            pub.publish("late/x", b"two")
            assert {got.get(timeout=5), got.get(timeout=5)} == {b"one", b"two"}
            pub.disconnect()
        finally:
            t.terminate()
            b2.stop()
    finally:
        t.terminate()


def test_websocket_clients_share_topics_with_tcp():
    """MQTT over WebSockets: a WS subscriber and a TCP publisher (and the reverse) on one broker;
    retained messages, QoS 1 and a 1 MB payload cross the frame layer."""
    b, port = start_broker_thread("127.0.0.1", 0, ws_port=0)
    try:
        ws_sub, q_ws = _client(b.ws_port)
        ws_sub.connect("127.0.0.1", b.ws_port, transport="websockets")
        tcp_sub, q_tcp = _client(port)
        tcp_sub.connect("127.0.0.1", port)
        ws_sub.subscribe("t/#")
        tcp_sub.subscribe("w/#")
        pub, _ = _client(port)
        pub.connect("127.0.0.1", port)
        big = bytes(range(256)) * 4096
        pub.publish("t/a", b"hello", qos=1, wait=True)
        pub.publish("t/big", big)
        assert q_ws.get(timeout=5)[:2] == ("t/a", b"hello")
        assert q_ws.get(timeout=5)[:2] == ("t/big", big)
        ws_sub.publish("w/x", b"from-ws", qos=1, wait=True)
        assert q_tcp.get(timeout=5)[:2] == ("w/x", b"from-ws")
        pub.publish("t/keep", b"kept", retain=True)
        late, q_late = _client(b.ws_port)
        late.connect("127.0.0.1", b.ws_port, transport="websockets")
        late.subscribe("t/keep")
        assert q_late.get(timeout=5) == ("t/keep", b"kept", True)
        for c in (ws_sub, tcp_sub, pub, late):
            c.disconnect()
    finally:
        b.stop()


def test_websocket_lwt_and_unknown_transport(monkeypatch):
    b, port = start_broker_thread("127.0.0.1", 0, ws_port=0)
    try:
        watcher, q = _client(port)
        watcher.connect("127.0.0.1", port)
        watcher.subscribe("lwt/#")
        c, _ = _client(b.ws_port)
        c.will_set("lwt/ws", b"(absent)")
        c.connect("127.0.0.1", b.ws_port, transport="websockets")
        c.sock.sock.shutdown(socket.SHUT_RDWR)    # abnormal: no DISCONNECT, no close frame
        assert q.get(timeout=5)[:2] == ("lwt/ws", b"(absent)")
        watcher.disconnect()
        from aiko_services_amd.message.message import MQTT
        monkeypatch.setenv("AIKO_MQTT_HOST", "127.0.0.1")
        monkeypatch.setenv("AIKO_MQTT_PORT", str(port))
        monkeypatch.setenv("AIKO_MQTT_TRANSPORT", "quic")
        with pytest.raises(ValueError):
            MQTT(message_handler=lambda *a: None)
        with pytest.raises(ValueError):
            MQTTClient().connect("127.0.0.1", port, transport="udp")
    finally:
        b.stop()
