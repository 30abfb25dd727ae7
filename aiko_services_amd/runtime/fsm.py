"""Tiny finite-state machine replacing the ``transitions`` package (reference ``main/state.py``).

A model declares ``states`` and ``transitions`` (list of {source, trigger, dest}); entering a
state calls ``model.on_enter_<state>(event_data)`` when defined.  ``transition()`` raises
``SystemExit`` on an invalid trigger, like the reference wrapper.
"""
from __future__ import annotations

from dataclasses import dataclass, field

__all__ = ["StateMachine", "EventData"]


@dataclass
class EventData:
    trigger: str
    source: str
    dest: str
    kwargs: dict = field(default_factory=dict)


class StateMachine:
    def __init__(self, model, initial="start"):
        self.model = model
        self._table = {}
        for t in model.transitions:
            sources = t["source"] if isinstance(t["source"], (list, tuple)) else [t["source"]]
            for s in sources:
                self._table[(s, t["trigger"])] = t["dest"]
        self.model.state = initial

    def get_state(self):
        return self.model.state

    def can(self, trigger) -> bool:
        return (self.model.state, trigger) in self._table

    def transition(self, action, parameters):
        key = (self.model.state, action)
        if key not in self._table:
            known = any(t["trigger"] == action for t in self.model.transitions)
            why = "invalid in this state" if known else "unknown action"
            raise SystemExit(f"Fatal error: StateMachine: state={self.model.state}, action={action} ({why})")
        source, dest = self.model.state, self._table[key]
        self.model.state = dest
        handler = getattr(self.model, f"on_enter_{dest}", None)
        if handler is not None:
            handler(EventData(action, source, dest, {"parameters": parameters}))
