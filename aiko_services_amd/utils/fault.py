"""Fault injection for tests and chaos runs ("a fault-injection hook (kill stage
rank / drop messages) for tests" — the reference has none).

Faults are configured programmatically (``inject(...)``) or from ``AIKO_FAULTS``, a ``;``
separated list:

* ``drop=P@FILTER``          drop published control messages whose topic matches the MQTT
                             filter FILTER with probability P (seeded, reproducible);
* ``error=ELEMENT@F1,F2``    ``process_frame`` of ELEMENT raises on those frame ids
                             (exercises the StreamEvent.ERROR -> destroy_stream path);
* ``delay=ELEMENT@SECONDS``  sleep before ELEMENT's ``process_frame`` (slow-stage / lease tests);
* ``kill=N``                 this process exits (``os._exit(KILL_EXIT_CODE)``) once N frames have
                             completed — a dead pipeline-parallel rank or worker;
* ``kill=N@rankR``           the same, only in the process whose ``RANK`` is R (one AIKO_FAULTS
                             for a whole multi-GPU launch: the other ranks ignore it).  The Nth
                             frame dies after its compute, before its response is sent.

The hot path pays one ``is None`` check per element when no fault is configured.
"""
from __future__ import annotations

from dataclasses import dataclass, field
import os
import random
import threading

__all__ = ["FaultPlan", "InjectedFault", "inject", "clear", "active", "KILL_EXIT_CODE"]

KILL_EXIT_CODE = 86


class InjectedFault(RuntimeError):
    """Raised inside an element by an ``error=`` fault."""


@dataclass
class FaultPlan:
    drop: list = field(default_factory=list)          # [(probability, topic filter)]
    errors: dict = field(default_factory=dict)        # element -> set of frame ids (None = all)
    delays: dict = field(default_factory=dict)        # element -> seconds
    kill_after_frames: int | None = None
    seed: int = 0
    dropped: int = 0
    frames_seen: int = 0

    def __post_init__(self):
        self._rng = random.Random(self.seed)
        self._lock = threading.Lock()

    # ---- message plane ------------------------------------------------------------------------
    def should_drop(self, topic: str) -> bool:
        from ..message.mqtt_codec import topic_matches
        for p, flt in self.drop:
            if topic_matches(flt, topic):
                with self._lock:
                    hit = self._rng.random() < p
                    if hit:
                        self.dropped += 1
                if hit:
                    return True
        return False

    # ---- frame plane --------------------------------------------------------------------------
    def before_element(self, element_name: str, frame_id):
        delay = self.delays.get(element_name)
        if delay:
            import time
            time.sleep(delay)
        frames = self.errors.get(element_name, ())
        if frames is None or (frames and _as_int(frame_id) in frames):
            raise InjectedFault(f"injected fault: {element_name} frame {frame_id}")

    def frame_completed(self):
        self.frames_seen += 1
        if self.kill_after_frames is not None and self.frames_seen >= self.kill_after_frames:
            os._exit(KILL_EXIT_CODE)


def _as_int(v):
    try:
        return int(v)
    except (TypeError, ValueError):
        return v


def parse(spec: str, seed: int = 0) -> FaultPlan:
    plan = FaultPlan(seed=seed)
    for item in filter(None, (s.strip() for s in spec.split(";"))):
        kind, _, arg = item.partition("=")
        what, _, where = arg.partition("@")
        if kind == "drop":
            plan.drop.append((float(what), where or "#"))
        elif kind == "error":
            plan.errors[what] = {int(f) for f in where.split(",") if f} if where else None
        elif kind == "delay":
            plan.delays[what] = float(where)
        elif kind == "kill":
            if where and where.startswith("rank"):
                if os.environ.get("RANK", "0") != where[4:]:
                    continue
            plan.kill_after_frames = int(what)
        else:
            raise ValueError(f"AIKO_FAULTS: unknown fault '{kind}' in '{item}'")
    return plan


_plan: FaultPlan | None = None


def active() -> FaultPlan | None:
    return _plan


def inject(spec: str | FaultPlan | None = None, seed: int = 0, **kw) -> FaultPlan:
    """``inject("drop=0.5@aiko/#;error=PE_2@3")`` or ``inject(errors={"PE_2": {3}})``."""
    global _plan
    if isinstance(spec, FaultPlan):
        _plan = spec
    else:
        _plan = parse(spec or "", seed)
        for k, v in kw.items():
            setattr(_plan, k, v)
    return _plan


def clear():
    global _plan
    _plan = None


if os.environ.get("AIKO_FAULTS"):
    inject(os.environ["AIKO_FAULTS"], seed=int(os.environ.get("AIKO_FAULTS_SEED", "0")))
