"""LifeCycleManager / LifeCycleClient (reference ``main/lifecycle.py:98-456``).

The manager creates clients through a subclass hook (``_lcm_create_client``), waits for each
client's ``(add_client <topic_path> <client_id>)`` handshake on its ``/control`` topic within
a handshake lease (30 s), then follows the client's ``lifecycle`` share with an ECConsumer and
its registrar presence through ActorDiscovery.  ``lcm_delete_client`` starts a deletion lease
after which the client is force-deleted.  Clients may be GPU worker processes
(``LifeCycleManagerGpuImpl`` pins one client per GPU through the ProcessManager).
"""
from __future__ import annotations

import os
import sys
from abc import abstractmethod

from ..runtime.actor import Actor
from ..runtime.connection import ConnectionState
from ..runtime.context import Interface, ServiceProtocolInterface, actor_args, compose_instance
from ..runtime.lease import Lease
from ..runtime.process import aiko
from ..runtime.service import ServiceFilter, ServiceProtocol
from ..utils.logger import get_log_level_name
from ..utils.sexpr import parse
from .process_manager import ProcessManager
from .share import ECConsumer, ECProducer
from .transport import ActorDiscovery

__all__ = ["LifeCycleManager", "LifeCycleManagerImpl", "LifeCycleClient", "LifeCycleClientImpl",
           "LifeCycleManagerTest", "LifeCycleManagerTestImpl", "LifeCycleClientTest",
           "LifeCycleClientTestImpl", "PROTOCOL_LIFECYCLE_MANAGER", "PROTOCOL_LIFECYCLE_CLIENT"]

_VERSION = 0
PROTOCOL_LIFECYCLE_MANAGER = f"{ServiceProtocol.AIKO}/lifecycle_manager:{_VERSION}"
PROTOCOL_LIFECYCLE_CLIENT = f"{ServiceProtocol.AIKO}/lifecycle_client:{_VERSION}"
DELETION_LEASE_TIME_DEFAULT = 30
HANDSHAKE_LEASE_TIME_DEFAULT = 30

_LOGGER = aiko.logger(__name__, log_level=os.environ.get("AIKO_LOG_LEVEL_LIFECYCLE", "INFO"))


class LifeCycleClientDetails:
    def __init__(self, client_id, topic_path, ec_consumer=None):
        self.client_id = client_id
        self.topic_path = topic_path
        self.ec_consumer = ec_consumer


class LifeCycleManager(ServiceProtocolInterface):
    Interface.default("LifeCycleManager", "aiko_services_amd.control.lifecycle.LifeCycleManagerImpl")

    @abstractmethod
    def lcm_create_client(self, parameters=None):
        """Create a client (bookkeeping here, creation in ``_lcm_create_client``)."""

    @abstractmethod
    def lcm_delete_client(self, client_id):
        """Delete a client (bookkeeping here, deletion in ``_lcm_delete_client``)."""


class LifeCycleManagerPrivate(Interface):
    Interface.default("LifeCycleManagerPrivate", "aiko_services_amd.control.lifecycle.LifeCycleManagerImpl")

    @abstractmethod
    def _lcm_create_client(self, client_id, lifecycle_manager_topic, parameters):
        pass

    @abstractmethod
    def _lcm_delete_client(self, client_id, force=False):
        pass

    @abstractmethod
    def _lcm_get_clients(self):
        pass

    @abstractmethod
    def _lcm_get_handshaking_clients(self):
        pass

    @abstractmethod
    def _lcm_lookup_client_state(self, client_id, client_state_key):
        pass


class LifeCycleManagerImpl(LifeCycleManager, LifeCycleManagerPrivate):
    def __init__(self, lifecycle_client_change_handler=None, ec_producer=None,
                 client_state_consumer_filter="(lifecycle)",
                 handshake_lease_time=HANDSHAKE_LEASE_TIME_DEFAULT,
                 deletion_lease_time=DELETION_LEASE_TIME_DEFAULT):
        self.lcm_lifecycle_client_change_handler = lifecycle_client_change_handler
        self.lcm_actor_discovery = None
        self.lcm_client_count = 0
        self.lcm_ec_producer = ec_producer
        self.lcm_client_state_consumer_filter = client_state_consumer_filter
        self.lcm_deletion_lease_time = deletion_lease_time
        self.lcm_deletion_leases: dict = {}
        self.lcm_handshake_lease_time = handshake_lease_time
        self.lcm_handshakes: dict = {}
        self.lcm_lifecycle_clients: dict = {}
        self.add_message_handler(self._lcm_topic_control_handler, self.topic_control)
        if self.lcm_ec_producer is not None:
            self.lcm_ec_producer.update("lifecycle_manager", {})
            self.lcm_ec_producer.update("lifecycle_manager_clients_active", 0)
            self.lcm_ec_producer.update("lifecycle_manager_clients_handshaking", 0)

    def _lcm_update_handshaking(self):
        if self.lcm_ec_producer is not None:
            self.lcm_ec_producer.update("lifecycle_manager_clients_handshaking", len(self.lcm_handshakes))

    def lcm_create_client(self, parameters=None):
        client_id = self.lcm_client_count
        self.lcm_client_count += 1
        self._lcm_create_client(client_id, self.topic_path, parameters or {})
        self.lcm_handshakes[client_id] = Lease(self.lcm_handshake_lease_time, client_id,
                                               lease_expired_handler=self._lcm_handshake_lease_expired_handler)
        self._lcm_update_handshaking()
        return client_id

    def lcm_delete_client(self, client_id):
        if client_id not in self.lcm_deletion_leases:
            self._lcm_delete_client(client_id)
            self.lcm_deletion_leases[client_id] = Lease(
                self.lcm_deletion_lease_time, client_id,
                lease_expired_handler=self._lcm_deletion_lease_expired_handler)

    def _lcm_topic_control_handler(self, _aiko, topic, payload_in):
        command, parameters = parse(payload_in)
        if command != "add_client" or len(parameters) != 2:
            return
        client_topic_path = parameters[0]
        try:
            client_id = int(parameters[1])
        except ValueError:
            return
        lease = self.lcm_handshakes.pop(client_id, None)
        if lease is None:
            _LOGGER.debug(f"LifeCycleClient {client_id} unknown")
            return
        lease.terminate()
        self._lcm_update_handshaking()
        if self.lcm_actor_discovery is None:
            self.lcm_actor_discovery = ActorDiscovery(self)
        self.lcm_actor_discovery.add_handler(self._lcm_service_change_handler,
                                             ServiceFilter([client_topic_path], "*", "*", "*", "*", "*"))
        ec_consumer = ECConsumer(self, client_id, {}, f"{client_topic_path}/control",
                                 self.lcm_client_state_consumer_filter)
        if self.lcm_lifecycle_client_change_handler:
            ec_consumer.add_handler(self.lcm_lifecycle_client_change_handler)
        self.lcm_lifecycle_clients[client_id] = LifeCycleClientDetails(client_id, client_topic_path, ec_consumer)
        if self.lcm_ec_producer is not None:
            self.lcm_ec_producer.update("lifecycle_manager_clients_active", len(self.lcm_lifecycle_clients))
            self.lcm_ec_producer.update(f"lifecycle_manager.{client_id}", client_topic_path)

    def _lcm_service_change_handler(self, command, service_details):
        if command != "remove" or not service_details:
            return
        topic_path = service_details[0]
        for details in list(self.lcm_lifecycle_clients.values()):
            if details.topic_path != topic_path:
                continue
            if details.ec_consumer:
                details.ec_consumer.terminate()
                details.ec_consumer = None
            client_id = details.client_id
            lease = self.lcm_deletion_leases.pop(client_id, None)
            if lease is not None:
                lease.terminate()
            del self.lcm_lifecycle_clients[client_id]
            if self.lcm_ec_producer is not None:
                self.lcm_ec_producer.update("lifecycle_manager_clients_active", len(self.lcm_lifecycle_clients))
                self.lcm_ec_producer.remove(f"lifecycle_manager.{client_id}")
            if self.lcm_lifecycle_client_change_handler:
                self.lcm_lifecycle_client_change_handler(client_id, "update", "lifecycle", "absent")

    def _lcm_deletion_lease_expired_handler(self, client_id):
        self.lcm_deletion_leases.pop(client_id, None)
        self._lcm_delete_client(client_id, force=True)

    def _lcm_handshake_lease_expired_handler(self, client_id):
        self.lcm_handshakes.pop(client_id, None)
        self._lcm_update_handshaking()
        self._lcm_delete_client(client_id)
        _LOGGER.debug(f"LifeCycleClient {client_id} handshake failed")

    def _lcm_get_clients(self):
        clients = self.lcm_ec_producer.get("lifecycle_manager") if self.lcm_ec_producer else None
        return {int(k): v for k, v in clients.items()} if clients else {}

    def _lcm_get_handshaking_clients(self):
        return list(self.lcm_handshakes)

    def _lcm_lookup_client_state(self, client_id, client_state_key):
        details = self.lcm_lifecycle_clients.get(client_id)
        if details and details.ec_consumer:
            return details.ec_consumer.cache.get(client_state_key)
        return None


class LifeCycleClient(ServiceProtocolInterface):
    Interface.default("LifeCycleClient", "aiko_services_amd.control.lifecycle.LifeCycleClientImpl")


class LifeCycleClientPrivate(Interface):
    Interface.default("LifeCycleClientPrivate", "aiko_services_amd.control.lifecycle.LifeCycleClientImpl")

    @abstractmethod
    def _lcc_get_lifecycle_manager_topic(self):
        pass

    @abstractmethod
    def _lcc_lifecycle_manager_change_handler(self, command, service_details):
        pass


class LifeCycleClientImpl(LifeCycleClient, LifeCycleClientPrivate):
    def __init__(self, context, client_id, lifecycle_manager_topic, ec_producer):
        self.lcc_added_to_lcm = False
        self.lcc_client_id = client_id
        self.lcc_ec_producer = ec_producer
        self.lcc_actor_discovery = None
        self.lcc_ec_producer.update("lifecycle_client.lifecycle_manager_topic", lifecycle_manager_topic)
        aiko.connection.add_handler(self._lcc_connection_handler)

    def _lcc_get_lifecycle_manager_topic(self):
        return self.lcc_ec_producer.get("lifecycle_client.lifecycle_manager_topic")

    def _lcc_connection_handler(self, connection, connection_state):
        if connection.is_connected(ConnectionState.REGISTRAR) and not self.lcc_added_to_lcm:
            lcm_topic = self._lcc_get_lifecycle_manager_topic()
            aiko.message.publish(f"{lcm_topic}/control", f"(add_client {self.topic_path} {self.lcc_client_id})")
            self.lcc_added_to_lcm = True
            self.lcc_actor_discovery = ActorDiscovery(self)
            self.lcc_actor_discovery.add_handler(self._lcc_lifecycle_manager_change_handler,
                                                 ServiceFilter([lcm_topic], "*", "*", "*", "*", "*"))

    def _lcc_lifecycle_manager_change_handler(self, command, service_details):
        pass


# ---- test / CLI implementations (reference lifecycle.py:292-456) -----------------------------

class LifeCycleManagerTest(Actor, LifeCycleManager):
    Interface.default("LifeCycleManagerTest", "aiko_services_amd.control.lifecycle.LifeCycleManagerTestImpl")


class LifeCycleManagerTestImpl(LifeCycleManagerTest):
    """Spawns ``client_count`` real client processes (optionally one per GPU)."""

    def __init__(self, context, client_count, gpus=None, handshake_lease_time=HANDSHAKE_LEASE_TIME_DEFAULT,
                 silent_clients=()):
        context.get_implementation("Actor").__init__(self, context)
        self.share.update({"source_file": f"v{_VERSION}⇒ {__file__}", "client_count": client_count})
        self.process_manager = ProcessManager()
        self.gpus = gpus
        self.silent_clients = set(silent_clients or ())   # self-test: clients that never handshake
        self.client_changes: list = []
        context.get_implementation("LifeCycleManager").__init__(self, self._lifecycle_client_change_handler,
                                                               self.ec_producer,
                                                               handshake_lease_time=handshake_lease_time)
        aiko.connection.add_handler(self._connection_state_handler)
        self._started = False

    def _lcm_create_client(self, client_id, lifecycle_manager_topic, parameters):
        gpu = None if not self.gpus else self.gpus[client_id % len(self.gpus)]
        if client_id in self.silent_clients:     # a process that never sends (add_client ...)
            self.process_manager.create(client_id, sys.executable,
                                        ["-c", "import time; time.sleep(3600)  # aiko_silent_client"])
            return
        self.process_manager.create(client_id, sys.executable,
                                    ["-m", "aiko_services_amd.control.lifecycle", "client", str(client_id),
                                     lifecycle_manager_topic], gpu=gpu)

    def _lcm_delete_client(self, client_id, force=False):
        self.process_manager.delete(client_id, kill=force)

    def _connection_state_handler(self, connection, connection_state):
        if connection.is_connected(ConnectionState.REGISTRAR) and not self._started:
            self._started = True
            for _ in range(int(self.share["client_count"])):
                self.lcm_create_client()

    def _lifecycle_client_change_handler(self, client_id, command, item_name, item_value):
        self.client_changes.append((client_id, command, item_name, item_value))
        _LOGGER.debug(f"LifeCycleClient: {client_id}: {command} {item_name} {item_value}")


class LifeCycleClientTest(Actor, LifeCycleClient):
    Interface.default("LifeCycleClientTest", "aiko_services_amd.control.lifecycle.LifeCycleClientTestImpl")


class LifeCycleClientTestImpl(LifeCycleClientTest):
    def __init__(self, context, client_id, lifecycle_manager_topic):
        context.get_implementation("Actor").__init__(self, context)
        self.share.update({"source_file": f"v{_VERSION}⇒ {__file__}", "client_id": client_id})
        context.get_implementation("LifeCycleClient").__init__(self, context, client_id,
                                                              lifecycle_manager_topic, self.ec_producer)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="LifeCycleManager / LifeCycleClient")
    sub = ap.add_subparsers(dest="cmd", required=True)
    m = sub.add_parser("manager")
    m.add_argument("client_count", nargs="?", type=int, default=1)
    m.add_argument("--gpus", default=None, help="comma separated GPU indices for the clients")
    m.add_argument("--handshake-lease", type=float, default=HANDSHAKE_LEASE_TIME_DEFAULT,
                   help="seconds a client has to send (add_client ...) before it is deleted")
    m.add_argument("--silent-clients", default="",
                   help="(self-test) comma separated client ids started as processes that never handshake")
    c = sub.add_parser("client")
    c.add_argument("client_id")
    c.add_argument("lifecycle_manager_topic")
    a = ap.parse_args(argv)
    if a.cmd == "manager":
        gpus = [int(g) for g in a.gpus.split(",")] if a.gpus else None
        init_args = actor_args("lifecycle_manager", protocol=PROTOCOL_LIFECYCLE_MANAGER)
        init_args["client_count"] = a.client_count
        init_args["gpus"] = gpus
        init_args["handshake_lease_time"] = a.handshake_lease
        init_args["silent_clients"] = [int(c) for c in a.silent_clients.split(",") if c.strip()]
        compose_instance(LifeCycleManagerTestImpl, init_args)
    else:
        init_args = actor_args("lifecycle_client", protocol=PROTOCOL_LIFECYCLE_CLIENT)
        init_args["client_id"] = a.client_id
        init_args["lifecycle_manager_topic"] = a.lifecycle_manager_topic
        compose_instance(LifeCycleClientTestImpl, init_args)
    aiko.process.run()


if __name__ == "__main__":
    main()
