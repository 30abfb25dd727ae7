"""Self-test services for the EC share and the ServicesCache (reference ``main/share.py:660-760``).

    python -m aiko_services_amd.tools.ec_test sc_test                 # dump registrar state
    python -m aiko_services_amd.tools.ec_test ec_test                 # run an ECProducerTest
    python -m aiko_services_amd.tools.ec_test ec_test PID [SID] [FILTER]  # consume its share

``ECProducerTest`` shares ``lifecycle / log_level / source_file / items.{key_1,key_2}`` and
applies live ``log_level`` edits; ``ECConsumerTest`` mirrors another process's share through an
``ECConsumer`` on ``{ns}/{host}/{pid}/{sid}/control`` and logs every change it sees.
"""
from __future__ import annotations

import argparse

from ..control.share import (ECConsumer, ECProducer, PROTOCOL_EC_CONSUMER, PROTOCOL_EC_PRODUCER,
                             services_cache_create_singleton)
from ..runtime.context import compose_instance, service_args
from ..runtime.process import aiko
from ..runtime.service import Service
from ..utils.configuration import get_hostname, get_namespace
from ..utils.logger import get_log_level_name

__all__ = ["ECConsumerTest", "ECProducerTest", "main"]

_VERSION = 0
SERVICE_TYPE_EC_CONSUMER = "ec_consumer_test"
SERVICE_TYPE_EC_PRODUCER = "ec_producer_test"
_LOGGER = aiko.logger(__name__)


class ECProducerTest(Service):
    def __init__(self, context):
        context.get_implementation("Service").__init__(self, context)
        self.share = {
            "lifecycle": "ready",
            "log_level": get_log_level_name(_LOGGER),
            "source_file": f"v{_VERSION}⇒ {__file__}",
            "items": {"key_1": ["item_1a", "item_1b"], "key_2": ["item_2a", "item_2b"]},
        }
        self.changes: list = []
        self.ec_producer = ECProducer(self, self.share)
        self.ec_producer.add_handler(self._ec_producer_change_handler)
        _LOGGER.info(f"ECProducer: topic path: {self.topic_path}")

    def _ec_producer_change_handler(self, command, item_name, item_value):
        self.changes.append((command, item_name, item_value))
        _LOGGER.info(f"ECProducer: {command} {item_name} {item_value}")
        if item_name == "log_level":
            _LOGGER.setLevel(str(item_value).upper())


class ECConsumerTest(Service):
    def __init__(self, context, ec_producer_pid, ec_producer_sid="1", filter="*",
                 ec_producer_topic_control=None):
        context.get_implementation("Service").__init__(self, context)
        self.share_producer = {
            "lifecycle": "ready",
            "log_level": get_log_level_name(_LOGGER),
            "source_file": f"v{_VERSION}⇒ {__file__}",
            "ec_producer_pid": ec_producer_pid,
            "ec_producer_sid": ec_producer_sid,
        }
        self.ec_producer = ECProducer(self, self.share_producer)
        self.share_consumer: dict = {}
        self.changes: list = []
        topic = ec_producer_topic_control or \
            f"{get_namespace()}/{get_hostname()}/{ec_producer_pid}/{ec_producer_sid}/control"
        self.ec_consumer = ECConsumer(self, 0, self.share_consumer, topic, filter)
        self.ec_consumer.add_handler(self._ec_consumer_change_handler)
        _LOGGER.info(f"ECConsumer: topic path: {self.topic_path} <- {topic}")

    def _ec_consumer_change_handler(self, client_id, command, item_name, item_value):
        self.changes.append((command, item_name, item_value))
        _LOGGER.info(f"ECConsumer: {client_id}: {command} {item_name} {item_value}")


def sc_test(timeout=10.0, history_limit=4):
    """Wait for the ServicesCache to load, log the running services and the history, exit."""
    cache = services_cache_create_singleton(aiko.process, True, history_limit=history_limit)
    _LOGGER.info("ServicesCache: Wait ready")
    if not cache.wait_ready(timeout):
        _LOGGER.warning(f"ServicesCache: not ready (state={cache.get_state()})")
    _LOGGER.info("ServicesCache: Services running")
    for details in cache.get_services():
        _LOGGER.info(f"{details}")
    _LOGGER.info("ServicesCache: Service history")
    for details in cache.get_history():
        _LOGGER.info(f"{details}")
    aiko.process.terminate()


def ec_test(ec_producer_pid=None, ec_producer_sid="1", filter="*"):
    tags = ["ec=true"]
    if ec_producer_pid:
        init_args = service_args(SERVICE_TYPE_EC_CONSUMER, None, None, PROTOCOL_EC_CONSUMER, tags)
        init_args.update(ec_producer_pid=ec_producer_pid, ec_producer_sid=ec_producer_sid,
                         filter=filter)
        service = compose_instance(ECConsumerTest, init_args)
    else:
        init_args = service_args(SERVICE_TYPE_EC_PRODUCER, None, None, PROTOCOL_EC_PRODUCER, tags)
        service = compose_instance(ECProducerTest, init_args)
    aiko.process.run(True)
    return service


def main(argv=None):
    ap = argparse.ArgumentParser(description="EC share / ServicesCache self tests")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("sc_test", help="Test Registrar Services Cache")
    s.add_argument("--timeout", type=float, default=10.0)
    e = sub.add_parser("ec_test", help="Test Eventual Consistency Producer and Consumer")
    e.add_argument("ec_producer_pid", nargs="?")
    e.add_argument("ec_producer_sid", nargs="?", default="1")
    e.add_argument("filter", nargs="?", default="*")
    a = ap.parse_args(argv)
    if a.cmd == "sc_test":
        sc_test(a.timeout)
    else:
        ec_test(a.ec_producer_pid, a.ec_producer_sid, a.filter)


if __name__ == "__main__":
    main()
