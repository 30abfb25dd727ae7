"""Data-plane bootstrap over the MQTT control plane.

SURVEY P1: the RCCL communicator's bootstrap is distributed over MQTT instead of a separate
launcher.  The process that plays rank 0 of a named group opens a free TCP port for
torch.distributed's store (through which RCCL exchanges its unique id), publishes
``(rendezvous group host port world_size generation)`` RETAINED on
``{namespace}/rendezvous/{group}``; the other members subscribe, read it, and all call
``init_process_group`` against that store.  Late joiners see the retained message; the
leader clears it after everyone connected (the store's own barrier), so a stale group is never
joined.  ``torchrun`` remains supported (``dist.init`` reads its environment variables).
"""
from __future__ import annotations

import datetime
import os
import socket
import threading
import time
import uuid

import torch
import torch.distributed as tdist

from ..message.mqtt_client import MQTTClient
from ..utils.configuration import get_namespace
from ..utils.sexpr import generate, parse
from . import dist as D

__all__ = ["rendezvous_topic", "rendezvous_init", "free_port", "store_address", "connect_store"]

_STORE_ADDR = None        # (host, port) of the group's TCPStore (rank 0 is its master)
_STORE = None             # this rank's handle on it (re-admission groups use raw keys on it)


def group_store():
    """This rank's TCPStore of the MQTT-bootstrapped group (None: not bootstrapped here)."""
    return _STORE


def store_address():
    """(host, port) of this process's group store, or None: what a restarted rank connects to
    (the rank-0 supervisor passes it in ``AIKO_REJOIN_STORE``)."""
    return _STORE_ADDR


def connect_store(address: str, timeout_s: float = 60.0):
    """A client of the running group's TCPStore (``host:port``), for a re-admitted rank."""
    host, port = address.rsplit(":", 1)
    return tdist.TCPStore(host, int(port), is_master=False, timeout=datetime.timedelta(seconds=timeout_s))


def rendezvous_topic(group: str) -> str:
    return f"{get_namespace()}/rendezvous/{group}"


def free_port(host="127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _advertised_host():
    host = os.environ.get("AIKO_RENDEZVOUS_HOST")
    if host:
        return host
    try:
        from ..utils.configuration import get_lan_ip_address
        return get_lan_ip_address()
    except Exception:
        return "127.0.0.1"


def rendezvous_init(group: str, rank: int, world_size: int, mqtt_host="127.0.0.1", mqtt_port=1883,
                    backend: str | None = None, timeout_s: float = 60.0) -> bool:
    """Join process group ``group`` as ``rank`` of ``world_size`` via the MQTT broker."""
    if world_size <= 1:
        return False
    backend = backend or ("nccl" if torch.cuda.is_available() else "gloo")
    topic = rendezvous_topic(group)
    got = {}
    ready = threading.Event()

    def on_message(_client, _userdata, msg):
        try:
            cmd, params = parse(msg.payload.decode() if isinstance(msg.payload, bytes) else msg.payload)
        except Exception:
            return
        if cmd == "rendezvous" and len(params) >= 4 and int(params[3]) == world_size:
            got.update(host=params[1], port=int(params[2]))
            ready.set()

    client = MQTTClient(client_id=f"aiko-rdv-{uuid.uuid4().hex[:8]}", on_message=on_message)
    client.connect(mqtt_host, mqtt_port)
    try:
        if rank == 0:
            host = _advertised_host()
            port = free_port("0.0.0.0" if host != "127.0.0.1" else "127.0.0.1")
            store = tdist.TCPStore(host, port, world_size, is_master=True, wait_for_workers=False,
                                   timeout=datetime.timedelta(seconds=timeout_s))
            global _STORE_ADDR
            _STORE_ADDR = (host, port)
            client.publish(topic, generate("rendezvous", [group, host, port, world_size, uuid.uuid4().hex[:8]]),
                           retain=True, qos=1, wait=True)
        else:
            client.subscribe(topic)
            if not ready.wait(timeout_s):
                raise TimeoutError(f"rendezvous {group}: no leader on {topic} after {timeout_s}s")
            store = tdist.TCPStore(got["host"], got["port"], world_size, is_master=False,
                                   timeout=datetime.timedelta(seconds=timeout_s))
        global _STORE
        _STORE = store
        kwargs = {}
        if backend == "nccl":
            dev = torch.device("cuda", D.local_rank() % max(1, torch.cuda.device_count()))
            torch.cuda.set_device(dev)
            kwargs["device_id"] = dev
        tdist.init_process_group(backend=backend, store=store, rank=rank, world_size=world_size,
                                 timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
        D._backend = backend
        D.barrier()
        if rank == 0:                     # everyone is in: retire the retained advertisement
            client.publish(topic, b"", retain=True, qos=1, wait=True)
        return True
    finally:
        time.sleep(0.05)
        client.disconnect()
