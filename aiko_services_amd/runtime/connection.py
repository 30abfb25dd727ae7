"""Connection state with observers (reference ``main/connection.py:12-46``).

States are ordered NONE < NETWORK < TRANSPORT < REGISTRAR; ``add_handler`` invokes the handler
immediately with the current state, then on every ``update_state``.
"""
from __future__ import annotations

import threading

__all__ = ["ConnectionState", "Connection"]


class ConnectionState:
    NONE = "NONE"
    NETWORK = "NETWORK"
    BOOTSTRAP = "BOOTSTRAP"
    TRANSPORT = "TRANSPORT"
    REGISTRAR = "REGISTRAR"

    states = [NONE, NETWORK, TRANSPORT, REGISTRAR]  # order matters

    @classmethod
    def index(cls, connection_state):
        return cls.states.index(connection_state)


class Connection:
    def __init__(self):
        self.connection_state = ConnectionState.NONE
        self.connection_state_handlers = []
        self._lock = threading.RLock()

    def add_handler(self, connection_state_handler):
        connection_state_handler(self, self.connection_state)
        with self._lock:
            if connection_state_handler not in self.connection_state_handlers:
                self.connection_state_handlers.append(connection_state_handler)

    def is_connected(self, connection_state):
        return ConnectionState.index(self.connection_state) >= ConnectionState.index(connection_state)

    def remove_handler(self, connection_state_handler):
        with self._lock:
            if connection_state_handler in self.connection_state_handlers:
                self.connection_state_handlers.remove(connection_state_handler)

    def update_state(self, connection_state):
        self.connection_state = connection_state
        with self._lock:
            handlers = list(self.connection_state_handlers)
        for handler in handlers:
            handler(self, connection_state)
