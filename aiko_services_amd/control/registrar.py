"""Registrar: the control plane's service directory (reference ``main/registrar.py:136-368``).

State machine ``start -> primary_search -> (secondary | primary)``.  The primary publishes a
retained ``(primary found <topic_path> <version> <time_started>)`` on ``{ns}/service/registrar``
and sets its last will to ``(primary absent)`` there, so every process learns of the registrar
(and of its failure) from the broker.  Protocol on ``{registrar}/in``:

* ``(add topic_path name protocol transport owner (tags))`` / ``(remove topic_path)``
* ``(share response_topic name protocol transport owner tags)`` -> ``(item_count N)`` + adds,
  then ``(sync response_topic)`` on ``{registrar}/out``
* ``(history response_topic count|*)`` -> removed services, most recent first

Split brain (two primaries, e.g. started together or after a partition): the oldest
``time_started`` wins, the other demotes itself to secondary (``_resolve_split_brain``).

Process failure: the broker delivers a process's LWT ``(absent)`` on ``{ns}/+/+/+/state``
and every service of that process is removed.  Fixes vs the reference: an explicit
``(remove topic)`` of a single service works (the reference iterated the topic string), and the
primary-search timeout carries jitter so concurrently started registrars do not all promote.
"""
from __future__ import annotations

import os
import random
import time
from collections import deque

from ..runtime import event
from ..runtime.context import Interface, compose_instance, service_args
from ..runtime.fsm import StateMachine
from ..runtime.process import aiko
from ..runtime.service import Service, ServiceFilter, ServiceProtocol, Services, ServiceTopicPath
from ..utils.configuration import get_namespace
from ..utils.logger import get_log_level_name
from ..utils.sexpr import generate, parse, parse_int
from .share import ECProducer

__all__ = ["Registrar", "RegistrarImpl", "REGISTRAR_PROTOCOL", "main"]

_VERSION = 2
SERVICE_TYPE = "registrar"
REGISTRAR_PROTOCOL = f"{ServiceProtocol.AIKO}/{SERVICE_TYPE}:{_VERSION}"
HISTORY_LIMIT_DEFAULT = 16
HISTORY_RING_BUFFER_SIZE = 4096
PRIMARY_SEARCH_TIMEOUT = float(os.environ.get("AIKO_REGISTRAR_SEARCH_TIMEOUT", 2.0))

_LOGGER = aiko.logger(__name__)


class StateMachineModel:
    states = ["start", "primary_search", "secondary", "primary"]
    transitions = [
        {"source": "start", "trigger": "initialize", "dest": "primary_search"},
        {"source": "primary_search", "trigger": "primary_found", "dest": "secondary"},
        {"source": "primary_search", "trigger": "primary_promotion", "dest": "primary"},
        {"source": "primary", "trigger": "primary_failed", "dest": "primary_search"},
        {"source": "secondary", "trigger": "primary_failed", "dest": "primary_search"},
        {"source": "secondary", "trigger": "primary_promotion", "dest": "primary"},
        {"source": "primary", "trigger": "primary_demotion", "dest": "secondary"},
    ]

    def __init__(self, service):
        self.service = service

    def on_enter_primary_search(self, event_data):
        self.service.ec_producer.update("lifecycle", "primary_search")
        jitter = random.uniform(0.0, 0.25 * PRIMARY_SEARCH_TIMEOUT)
        event.add_timer_handler(self.primary_search_timer, PRIMARY_SEARCH_TIMEOUT + jitter)

    def primary_search_timer(self):
        event.remove_timer_handler(self.primary_search_timer)
        if self.service.state_machine.get_state() == "primary_search":
            self.service.state_machine.transition("primary_promotion", None)

    def on_enter_secondary(self, event_data):
        self.service.ec_producer.update("lifecycle", "secondary")

    def on_enter_primary(self, event_data):
        self.service.ec_producer.update("lifecycle", "primary")
        # clear the retained boot message, install our LWT, announce ourselves (retained)
        aiko.message.publish(aiko.TOPIC_REGISTRAR_BOOT, "", retain=True)
        aiko.process.set_last_will_and_testament(aiko.TOPIC_REGISTRAR_BOOT, "(primary absent)", True)
        self.service.announce()


class Registrar(Service):
    Interface.default("Registrar", "aiko_services_amd.control.registrar.RegistrarImpl")


class RegistrarImpl(Registrar):
    def __init__(self, context):
        context.get_implementation("Service").__init__(self, context)
        self.state_machine = StateMachine(StateMachineModel(self))
        self.history: deque = deque(maxlen=HISTORY_RING_BUFFER_SIZE)
        self.services = Services()
        self.share = {
            "lifecycle": "start",
            "log_level": get_log_level_name(_LOGGER),
            "source_file": f"v{_VERSION}⇒ {__file__}",
            "service_count": 0,
        }
        self.ec_producer = ECProducer(self, self.share)
        self.ec_producer.add_handler(self._ec_producer_change_handler)
        self.add_message_handler(self._service_state_handler, f"{get_namespace()}/+/+/+/state")
        self.add_message_handler(self._topic_in_handler, self.topic_in)
        self.set_registrar_handler(self._registrar_handler)
        self.state_machine.transition("initialize", None)

    def _ec_producer_change_handler(self, command, item_name, item_value):
        if item_name == "log_level":
            try:
                _LOGGER.setLevel(str(item_value).upper())
            except ValueError:
                pass

    def announce(self):
        payload = f"(primary found {self.topic_path} {_VERSION} {self.time_started})"
        aiko.message.publish(aiko.TOPIC_REGISTRAR_BOOT, payload, retain=True)

    def _registrar_handler(self, action, registrar):
        state = self.state_machine.get_state()
        if action == "found":
            if registrar and registrar.get("topic_path") == self.topic_path:
                return
            if state == "primary_search":
                self.state_machine.transition("primary_found", None)
            elif state == "primary":
                self._resolve_split_brain(registrar or {})
        elif action == "absent":
            if state == "primary_search":
                self.state_machine.transition("primary_promotion", None)
            elif state in ("primary", "secondary"):
                self.services = Services()
                self.ec_producer.update("service_count", 0)
                self.state_machine.transition("primary_failed", None)

    def _resolve_split_brain(self, other):
        """Another registrar announced itself while this one is primary (two promoted at once,
        or a partition healed; the reference ignores it, main/registrar.py:139-188): the OLDEST
        (time_started, then topic path) stays primary.  The loser becomes secondary and gives
        back the "(primary absent)" will (its death must not unseat the winner); the winner
        re-announces, so the retained boot message and every process's registrar end up on it."""
        try:
            theirs = (float(other.get("timestamp")), str(other.get("topic_path")))
        except (TypeError, ValueError):
            return
        if theirs < (float(self.time_started), self.topic_path):
            _LOGGER.info(f"Registrar {theirs[1]} is older: demoted to secondary")
            self.state_machine.transition("primary_demotion", None)
            aiko.process.set_last_will_and_testament(aiko.topic_lwt, aiko.payload_lwt, False)
        else:
            self.announce()

    def _service_state_handler(self, _aiko, topic, payload_in):
        command, _ = parse(payload_in)
        if command == "absent" and topic.endswith("/state"):
            self._service_remove(topic[:-len("/state")])

    @staticmethod
    def _details_payload(d, with_times=False):
        tags = " ".join(d["tags"]) if isinstance(d["tags"], list) else str(d["tags"])
        payload = (f"(add {d['topic_path']} {d['name']} {d['protocol']} {d['transport']} "
                   f"{d['owner']} ({tags})")
        if with_times:
            payload += f" {d['time_add']} {d['time_remove']}"
        return payload + ")"

    def _topic_in_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command == "add" and len(parameters) == 6:
            self._service_add(*parameters, payload_in)
        elif command == "remove" and len(parameters) == 1:
            self._service_remove(parameters[0])
        elif command == "history" and len(parameters) == 2:
            response_topic = parameters[0]
            count = HISTORY_LIMIT_DEFAULT if parameters[1] == "*" else parse_int(parameters[1])
            count = min(count, len(self.history))
            aiko.message.publish(response_topic, f"(item_count {count})")
            for d in list(self.history)[:count]:
                aiko.message.publish(response_topic, self._details_payload(d, with_times=True))
        elif command == "share" and len(parameters) == 6:
            response_topic, name, protocol, transport, owner, tags = parameters
            filter_ = ServiceFilter("*", name, protocol, transport, owner, tags)
            matched = self.services.filter_by_attributes(filter_)
            aiko.message.publish(response_topic, f"(item_count {matched.count})")
            for d in matched:
                aiko.message.publish(response_topic, self._details_payload(d))
            aiko.message.publish(self.topic_out, f"(sync {response_topic})")

    def _service_add(self, topic_path, name, protocol, transport, owner, tags, payload_out):
        if self.services.get_service(topic_path):
            return
        self.services.add_service(topic_path, {
            "topic_path": topic_path, "name": name, "protocol": protocol, "transport": transport,
            "owner": owner, "tags": tags if isinstance(tags, list) else [tags],
            "time_add": time.time(), "time_remove": 0,
        })
        self.ec_producer.update("service_count", self.services.count)
        aiko.message.publish(self.topic_out, payload_out)

    def _service_remove(self, topic_path):
        stp = ServiceTopicPath.parse(topic_path)
        if not stp:
            return
        if str(stp.service_id) == "0":   # a whole process terminated
            process_tp, _ = ServiceTopicPath.topic_paths(topic_path)
            topic_paths = self.services.get_process_services(process_tp)
        else:
            topic_paths = [topic_path]
        for tp in list(topic_paths):
            d = self.services.get_service(tp)
            if d:
                d["time_remove"] = time.time()
                self.history.appendleft(d)
                self.services.remove_service(tp)
                self.ec_producer.update("service_count", self.services.count)
                aiko.message.publish(self.topic_out, f"(remove {tp})")


def create_registrar():
    init_args = service_args(SERVICE_TYPE, None, None, REGISTRAR_PROTOCOL, ["ec=true"])
    return compose_instance(RegistrarImpl, init_args)


def main(argv=None):
    """``aiko_registrar``: run a registrar service (needs a reachable broker)."""
    import argparse
    ap = argparse.ArgumentParser(description="Registrar Service")
    ap.parse_args(argv)
    create_registrar()
    aiko.process.run(True)


if __name__ == "__main__":
    main()

