"""Storage actor: SQLite-backed key/value store plus request/response helpers
(reference ``main/storage.py:49-140``, where the store was a stub).

Commands on ``{storage}/in``: ``(put key value)``, ``(delete key)``, ``(get response_topic
key)``, ``(list response_topic [prefix])`` and the reference's ``(test_command p)`` /
``(test_request response_topic request)``.  Responses use the ``(item_count N)`` + N items
convention.  ``do_command`` / ``do_request`` discover the storage actor through the registrar
and run a command / a request-response exchange against it.
"""
from __future__ import annotations

import sqlite3
from abc import abstractmethod

from ..control.transport import ActorDiscovery, get_actor_mqtt
from ..runtime import event
from ..runtime.actor import Actor
from ..runtime.context import Interface, actor_args, compose_instance
from ..runtime.process import aiko
from ..runtime.service import ServiceFilter, ServiceProtocol
from ..utils.sexpr import generate, parse

__all__ = ["Storage", "StorageImpl", "PROTOCOL", "do_command", "do_request", "main"]

_VERSION = 0
ACTOR_TYPE = "storage"
PROTOCOL = f"{ServiceProtocol.AIKO}/{ACTOR_TYPE}:{_VERSION}"
TOPIC_RESPONSE = f"{aiko.topic_out}/storage_response"


class Storage(Actor):
    Interface.default("Storage", "aiko_services_amd.tools.storage.StorageImpl")

    @abstractmethod
    def put(self, key, value):
        pass

    @abstractmethod
    def get(self, topic_path_response, key):
        pass

    @abstractmethod
    def delete(self, key):
        pass

    @abstractmethod
    def list(self, topic_path_response, prefix=""):
        pass

    @abstractmethod
    def test_command(self, parameter):
        pass

    @abstractmethod
    def test_request(self, topic_path_response, request):
        pass


class StorageImpl(Storage):
    def __init__(self, context, database_pathname=":memory:"):
        context.get_implementation("Actor").__init__(self, context)
        self.connection = sqlite3.connect(database_pathname, check_same_thread=False)
        self.connection.execute("create table if not exists kv (key text primary key, value text)")
        self.connection.commit()
        self.share["database_pathname"] = database_pathname
        self.share["source_file"] = f"v{_VERSION}⇒ {__file__}"
        self.commands = []

    def put(self, key, value):
        self.connection.execute("insert or replace into kv values (?, ?)", (str(key), str(value)))
        self.connection.commit()

    def get(self, topic_path_response, key):
        row = self.connection.execute("select value from kv where key = ?", (str(key),)).fetchone()
        items = [] if row is None else [generate("item", [key, row[0]])]
        self._respond(topic_path_response, items)

    def delete(self, key):
        self.connection.execute("delete from kv where key = ?", (str(key),))
        self.connection.commit()

    def list(self, topic_path_response, prefix=""):
        rows = self.connection.execute("select key, value from kv where key like ? order by key",
                                       (f"{prefix}%",)).fetchall()
        self._respond(topic_path_response, [generate("item", [k, v]) for k, v in rows])

    def _respond(self, topic, items):
        aiko.message.publish(topic, f"(item_count {len(items)})")
        for item in items:
            aiko.message.publish(topic, item)

    def test_command(self, parameter):
        self.commands.append(parameter)
        self.logger.info(f"Command: test_command({parameter})")

    def test_request(self, topic_path_response, request):
        self._respond(topic_path_response, [f"({request})"])


def do_command(actor_interface, command_handler, terminate=True, protocol=PROTOCOL):
    """Discover the actor implementing ``protocol``, then run ``command_handler(proxy)``."""
    def waiting():
        event.remove_timer_handler(waiting)
        print(f"Waiting for {protocol}")

    def discovered(command, details):
        if command == "add" and details:
            event.remove_timer_handler(waiting)
            command_handler(get_actor_mqtt(f"{details[0]}/in", actor_interface))
            if terminate:
                aiko.process.terminate()

    ActorDiscovery(aiko.process).add_handler(discovered, ServiceFilter("*", "*", protocol, "*", "*", "*"))
    event.add_timer_handler(waiting, 0.5)
    aiko.process.run()


def do_request(actor_interface, request_handler, response_handler, protocol=PROTOCOL):
    state = {"count": 0, "received": 0, "items": []}

    def on_response(_aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command == "item_count" and len(parameters) == 1:
            state.update(count=int(parameters[0]), received=0, items=[])
            if state["count"] == 0:
                response_handler([])
        elif state["received"] < state["count"]:
            state["items"].append((command, parameters))
            state["received"] += 1
            if state["received"] == state["count"]:
                response_handler(state["items"])

    aiko.process.add_message_handler(on_response, TOPIC_RESPONSE)
    do_command(actor_interface, request_handler, terminate=False, protocol=protocol)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Storage actor")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start")
    s.add_argument("database_pathname", nargs="?", default="aiko_storage.db")
    sub.add_parser("test_command")
    r = sub.add_parser("test_request")
    r.add_argument("request")
    a = ap.parse_args(argv)
    if a.cmd == "start":
        init_args = actor_args(ACTOR_TYPE, protocol=PROTOCOL, tags=["ec=true"])
        init_args["database_pathname"] = a.database_pathname
        compose_instance(StorageImpl, init_args).run()
    elif a.cmd == "test_command":
        do_command(Storage, lambda storage: storage.test_command("hello"))
    else:
        def handler(response):
            print(f"Response: {response}")
            aiko.process.terminate()
        do_request(Storage, lambda storage: storage.test_request(TOPIC_RESPONSE, a.request), handler)


if __name__ == "__main__":
    main()
