"""``aiko_mqtt``: broker / publish / subscribe helpers (mosquitto, mosquitto_pub and
mosquitto_sub are not part of the target environment; reference ``scripts/system_start.sh``,
``scripts/mqtt_sub_all.sh``).

    python -m aiko_services_amd.tools.mqtt broker [--port 1883]
    python -m aiko_services_amd.tools.mqtt pub TOPIC PAYLOAD [--retain]
    python -m aiko_services_amd.tools.mqtt sub [TOPIC ...] [--count N] [--timeout S]
    python -m aiko_services_amd.tools.mqtt reset          # clear the retained registrar topic
"""
from __future__ import annotations

import argparse
import sys
import threading
import time

from ..message.mqtt_client import MQTTClient
from ..utils.configuration import get_mqtt_host, get_namespace

__all__ = ["main"]


def _connect(on_message=None):
    _up, host, port = get_mqtt_host()
    c = MQTTClient(on_message=on_message)
    c.connect(host, port)
    return c


def main(argv=None):
    ap = argparse.ArgumentParser(prog="aiko_mqtt")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("broker")
    b.add_argument("--host", default="0.0.0.0")
    b.add_argument("--port", type=int, default=1883)
    p = sub.add_parser("pub")
    p.add_argument("topic")
    p.add_argument("payload")
    p.add_argument("--retain", action="store_true")
    s = sub.add_parser("sub")
    s.add_argument("topics", nargs="*")
    s.add_argument("--count", type=int, default=0)
    s.add_argument("--timeout", type=float, default=0.0)
    sub.add_parser("reset")
    a = ap.parse_args(argv)

    if a.cmd == "broker":
        from ..message.mqtt_broker import Broker
        broker = Broker(a.host, a.port)
        print(f"aiko MQTT broker on {a.host}:{broker.bind()}", flush=True)
        broker.serve_forever()
        return 0
    if a.cmd == "pub":
        c = _connect()
        c.publish(a.topic, a.payload, retain=a.retain, qos=1, wait=True)
        c.disconnect()
        return 0
    if a.cmd == "reset":
        c = _connect()
        c.publish(f"{get_namespace()}/service/registrar", b"", retain=True, qos=1, wait=True)
        c.disconnect()
        return 0
    seen = [0]
    done = threading.Event()

    def on_message(_c, _u, msg):
        payload = msg.payload.decode(errors="replace") if isinstance(msg.payload, bytes) else msg.payload
        print(f"{msg.topic} {payload}", flush=True)
        seen[0] += 1
        if a.count and seen[0] >= a.count:
            done.set()

    c = _connect(on_message)
    c.subscribe(a.topics or [f"{get_namespace()}/#"])
    deadline = time.time() + a.timeout if a.timeout else None
    try:
        while not done.is_set() and (deadline is None or time.time() < deadline):
            done.wait(0.1)
    except KeyboardInterrupt:
        pass
    c.disconnect()
    return 0


if __name__ == "__main__":
    sys.exit(main())
