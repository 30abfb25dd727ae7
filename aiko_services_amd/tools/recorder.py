"""Recorder service: keeps the recent log records of every process (reference ``main/recorder.py``).

Subscribes to ``{namespace}/+/+/+/log`` (or a given filter), keeps a ring buffer of records per
log topic inside an LRU of topics, and exposes the latest record per topic through its
ECProducer as ``lru_cache.<topic>`` so a dashboard can follow it.  Records keep their text;
S-expression delimiters are made safe the way the reference does (parentheses -> braces).
"""
from __future__ import annotations

from collections import deque

from ..control.share import ECProducer
from ..runtime.context import Interface, compose_instance, service_args
from ..runtime.process import aiko
from ..runtime.service import Service, ServiceProtocol
from ..utils.configuration import get_namespace
from ..utils.logger import get_log_level_name
from ..utils.misc import LRUCache

__all__ = ["Recorder", "RecorderImpl", "PROTOCOL", "main"]

_VERSION = 0
SERVICE_TYPE = "recorder"
PROTOCOL = f"{ServiceProtocol.AIKO}/{SERVICE_TYPE}:{_VERSION}"
LRU_CACHE_SIZE = 128
RING_BUFFER_SIZE = 128

_LOGGER = aiko.logger(__name__)


class Recorder(Service):
    Interface.default("Recorder", "aiko_services_amd.tools.recorder.RecorderImpl")


class RecorderImpl(Recorder):
    def __init__(self, context, topic_path_filter, lru_cache_size=LRU_CACHE_SIZE,
                 ring_buffer_size=RING_BUFFER_SIZE):
        context.get_implementation("Service").__init__(self, context)
        self.lru_cache = LRUCache(lru_cache_size)
        self.ring_buffer_size = ring_buffer_size
        self.share = {
            "lifecycle": "ready",
            "log_level": get_log_level_name(_LOGGER),
            "source_file": f"v{_VERSION}⇒ {__file__}",
            "lru_cache": {},
            "lru_cache_size": lru_cache_size,
            "ring_buffer_size": ring_buffer_size,
            "topic_path_filter": topic_path_filter,
        }
        self.ec_producer = ECProducer(self, self.share)
        self.add_message_handler(self.recorder_handler, topic_path_filter)

    def recorder_handler(self, _aiko, topic, payload_in):
        ring = self.lru_cache.get(topic)
        if ring is None:
            ring = deque(maxlen=self.ring_buffer_size)
            evicted = None
            if len(self.lru_cache) >= self.lru_cache.size:
                evicted = next(iter(self.lru_cache.cache))
            self.lru_cache.put(topic, ring)
            if evicted is not None and evicted not in self.lru_cache:
                self.ec_producer.remove(f"lru_cache.{evicted}")
        record = str(payload_in).replace("(", "{").replace(")", "}")
        ring.append(record)
        self.ec_producer.update(f"lru_cache.{topic}", record)

    def get_records(self, topic):
        ring = self.lru_cache.get(topic)
        return list(ring) if ring else []


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="Recorder Service")
    ap.add_argument("topic_path_filter", nargs="?", default=f"{get_namespace()}/+/+/+/log")
    a = ap.parse_args(argv)
    init_args = service_args(SERVICE_TYPE, None, None, PROTOCOL, ["ec=true"])
    init_args["topic_path_filter"] = a.topic_path_filter
    compose_instance(RecorderImpl, init_args)
    aiko.process.run()


if __name__ == "__main__":
    main()
