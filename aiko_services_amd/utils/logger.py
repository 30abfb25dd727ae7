"""Logging helpers (reference ``utilities/logger.py``).

``get_logger(name)`` names the logger after the last dotted component, upper-cased, with the
reference's line format.  ``LoggingHandlerMQTT`` buffers up to 128 records until the process
reaches the TRANSPORT connection state, then publishes every record to the process log topic
(and echoes to the console when the option is ``all``).  Unlike the reference, repeated
``get_logger`` calls do not stack duplicate handlers.
"""
from __future__ import annotations

import logging
import os
import sys
from collections import deque

__all__ = ["DEBUG", "INFO", "get_level_name", "get_log_level_name", "get_logger",
           "LoggingHandlerMQTT", "print_error"]

DEBUG = logging.DEBUG
INFO = logging.INFO
RING_BUFFER_SIZE = 128

_LEVEL_NAMES = {
    0: "LOG_LEVEL_NOTSET",
    logging.DEBUG: "DEBUG",
    logging.INFO: "INFO",
    logging.WARNING: "WARNING",
    logging.ERROR: "ERROR",
    logging.CRITICAL: "CRITICAL",
}

LOG_FORMAT = "%(asctime)s.%(msecs)03d %(levelname) 8s %(name)18s %(message)s"
LOG_FORMAT_DATETIME = "%Y-%m-%d_%H:%M:%S"


def get_log_level_name(logger) -> str:
    return _LEVEL_NAMES.get(logger.level, str(logger.level))


get_level_name = get_log_level_name


def _normalise_level(level):
    if level is None or level == "":
        level = os.environ.get("AIKO_LOG_LEVEL", logging.INFO)
    if isinstance(level, str):
        level = level.upper()
        if level.isdigit():
            level = int(level)
    return level or logging.INFO


def get_logger(name: str, log_level=None, logging_handler=None) -> logging.Logger:
    name = name.rpartition(".")[-1].upper()
    logger = logging.getLogger(name)
    if logging_handler is None and not logger.handlers:
        logging_handler = logging.StreamHandler()
    if logging_handler is not None:
        logging_handler.setFormatter(logging.Formatter(LOG_FORMAT, datefmt=LOG_FORMAT_DATETIME))
        # one aiko handler per logger (the MQTT handler echoes to the console itself)
        for h in list(logger.handlers):
            logger.removeHandler(h)
        logger.addHandler(logging_handler)
    logger.propagate = False
    try:
        logger.setLevel(_normalise_level(log_level))
    except (ValueError, TypeError):
        logger.setLevel(logging.INFO)
    return logger


def print_error(*args, **kwargs):
    print(*args, file=sys.stderr, **kwargs)


class LoggingHandlerMQTT(logging.Handler):
    """Publish log records on the process log topic once the transport is connected."""

    def __init__(self, aiko, topic, option="all", ring_buffer_size=RING_BUFFER_SIZE):
        super().__init__()
        self.aiko = aiko
        self.console_flag = option == "all"
        self.topic = topic
        self.ready = False
        self.ring_buffer: deque = deque(maxlen=ring_buffer_size)
        aiko.connection.add_handler(self._connection_state_handler)

    def _connection_state_handler(self, connection, connection_state):
        from ..runtime.connection import ConnectionState
        if connection.is_connected(ConnectionState.TRANSPORT):
            self.ready = True
            while self.ring_buffer:
                self.aiko.message.publish(self.topic, self.ring_buffer.popleft())
        else:
            self.ready = False

    def emit(self, record):
        try:
            payload = self.format(record)
            if self.console_flag:
                try:
                    print(payload, flush=True)
                except BrokenPipeError:
                    pass
            if self.ready and self.aiko.message is not None:
                self.aiko.message.publish(self.topic, payload)
            else:
                self.ring_buffer.append(payload)
        except Exception:
            self.handleError(record)
