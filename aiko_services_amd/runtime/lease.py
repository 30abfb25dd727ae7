"""Lease: timer-driven expiry with optional automatic extension (reference ``main/lease.py``).

``Lease(lease_time, lease_uuid, lease_expired_handler, lease_extend_handler,
automatic_extend)`` fires ``lease_expired_handler(lease_uuid)`` after ``lease_time`` unless
``extend()`` is called; with ``automatic_extend`` it extends itself every 0.8 x lease_time and
calls ``lease_extend_handler(lease_time, lease_uuid)`` (used by EC consumers to renew shares).
"""
from __future__ import annotations

from . import event

__all__ = ["Lease", "LEASE_EXTEND_TIME_FACTOR"]

LEASE_EXTEND_TIME_FACTOR = 0.8


class Lease:
    def __init__(self, lease_time, lease_uuid, lease_expired_handler=None,
                 lease_extend_handler=None, automatic_extend=False):
        self.lease_time = lease_time
        self.lease_uuid = lease_uuid
        self.lease_expired_handler = lease_expired_handler
        self.lease_extend_handler = lease_extend_handler
        self.automatic_extend = automatic_extend
        self.expired = False
        self.terminated = False
        self._deadline = event.engine.clock() + lease_time
        event.add_timer_handler(self._lease_expired_timer, lease_time)
        if automatic_extend:
            event.add_timer_handler(self.extend, lease_time * LEASE_EXTEND_TIME_FACTOR)

    def extend(self, lease_time=None):
        if self.terminated:
            return
        if lease_time and lease_time != self.lease_time:
            self.lease_time = lease_time
            event.remove_timer_handler(self._lease_expired_timer)
            event.add_timer_handler(self._lease_expired_timer, self.lease_time)
        # lazy: only the deadline moves (a stream lease is extended by every frame); the timer
        # re-arms itself for the rest when it fires early
        self._deadline = event.engine.clock() + self.lease_time
        if self.lease_extend_handler:
            self.lease_extend_handler(self.lease_time, self.lease_uuid)

    def _lease_expired_timer(self):
        event.remove_timer_handler(self._lease_expired_timer)
        left = self._deadline - event.engine.clock()
        if left > 1e-3 and not self.terminated:
            event.add_timer_handler(self._lease_expired_timer, left)
            return
        if self.automatic_extend:
            event.remove_timer_handler(self.extend)
        self.expired = True
        self.terminated = True
        if self.lease_expired_handler:
            self.lease_expired_handler(self.lease_uuid)

    def terminate(self):
        if self.terminated:
            return
        self.terminated = True
        event.remove_timer_handler(self._lease_expired_timer)
        if self.automatic_extend:
            event.remove_timer_handler(self.extend)
