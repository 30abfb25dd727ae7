"""Frame-span tracing with Chrome-trace (``chrome://tracing`` / Perfetto) export.

The reference times every local ``process_frame`` into ``frame.metrics`` and has no trace
export, GPU timing or communication accounting (reference
``main/pipeline.py:1031,1052,1069-1070``, ``elements/pipeline/elements.py:133-149``).  Here the
same hook points also feed a process-wide ``Tracer``:

* host spans: one per frame (``frame``) and one per element invocation (``element``), with the
  stream and frame ids as arguments, on the thread that ran them;
* GPU spans: a pair of HIP events around an element's work on its own HIP stream; the events are
  resolved only at export time (``elapsed_time`` against an anchor event recorded when the tracer
  was enabled), so tracing never synchronises the device in the hot path;
* communication spans / counters from ``parallel.dist`` (bytes per collective);
* counters (``ph: "C"``) such as queue depth or frames in flight.

Enable with ``AIKO_TRACE=/path/trace.json`` (written at exit) or ``enable_tracing(path)``; the
event buffer is a bounded ring (``AIKO_TRACE_EVENTS``, default 1,000,000) so a long-running
service keeps the most recent window.
"""
from __future__ import annotations

import atexit
from collections import deque
import json
import os
import threading
import time

__all__ = ["Tracer", "get_tracer", "enable_tracing", "disable_tracing", "tracing_enabled"]


class Tracer:
    def __init__(self, path: str | None = None, capacity: int = 1_000_000):
        self.path = path
        self.events: deque = deque(maxlen=capacity)
        self._gpu: deque = deque(maxlen=capacity)      # (name, cat, start_event, end_event, args, tid)
        self._lock = threading.Lock()
        self._pid = os.getpid()
        self._t0 = time.perf_counter()
        self._anchor = None                             # (cuda event, host us) for GPU spans

    # ---- time base -----------------------------------------------------------------------
    def now_us(self) -> float:
        return (time.perf_counter() - self._t0) * 1e6

    def to_us(self, perf_counter_s: float) -> float:
        return (perf_counter_s - self._t0) * 1e6

    # ---- recording ---------------------------------------------------------------------------
    def span(self, name: str, start_s: float, end_s: float, cat: str = "element", args=None, tid=None):
        """Complete event from two ``time.perf_counter()`` readings."""
        ev = {"name": name, "cat": cat, "ph": "X", "ts": self.to_us(start_s),
              "dur": max(0.0, (end_s - start_s) * 1e6), "pid": self._pid,
              "tid": tid if tid is not None else threading.get_ident()}
        if args:
            ev["args"] = args
        self.events.append(ev)

    def instant(self, name: str, cat: str = "event", args=None):
        ev = {"name": name, "cat": cat, "ph": "i", "s": "t", "ts": self.now_us(), "pid": self._pid,
              "tid": threading.get_ident()}
        if args:
            ev["args"] = args
        self.events.append(ev)

    def counter(self, name: str, values: dict):
        self.events.append({"name": name, "ph": "C", "ts": self.now_us(), "pid": self._pid,
                            "args": dict(values)})

    def gpu_span(self, name: str, start_event, end_event, cat: str = "gpu", args=None, stream_name="hip"):
        """Record a pair of timing-enabled ``torch.cuda.Event``s (already recorded on a stream)."""
        if self._anchor is None:
            self._make_anchor()
        self._gpu.append((name, cat, start_event, end_event, args, stream_name))

    def _make_anchor(self):
        import torch
        with self._lock:
            if self._anchor is not None:
                return
            torch.cuda.synchronize()
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            ev.synchronize()
            self._anchor = (ev, self.now_us())

    # ---- export ----------------------------------------------------------------------------
    def _resolve_gpu(self):
        out = []
        if self._anchor is None or not self._gpu:
            return out
        anchor, host_us = self._anchor
        tids = {}
        for name, cat, s, e, args, stream_name in list(self._gpu):
            try:
                e.synchronize()
                ts = host_us + anchor.elapsed_time(s) * 1e3
                dur = s.elapsed_time(e) * 1e3
            except RuntimeError:
                continue
            tid = tids.setdefault(stream_name, f"gpu:{stream_name}")
            ev = {"name": name, "cat": cat, "ph": "X", "ts": ts, "dur": dur, "pid": self._pid, "tid": tid}
            if args:
                ev["args"] = args
            out.append(ev)
        return out

    def chrome_events(self) -> list:
        evs = list(self.events) + self._resolve_gpu()
        evs.append({"name": "process_name", "ph": "M", "pid": self._pid,
                    "args": {"name": f"aiko {os.environ.get('RANK', '0')}:{self._pid}"}})
        return evs

    def export(self, path: str | None = None) -> str:
        path = path or self.path
        if not path:
            raise ValueError("Tracer.export: no path")
        if "{rank}" in path:
            path = path.replace("{rank}", os.environ.get("RANK", "0"))
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump({"traceEvents": self.chrome_events(), "displayTimeUnit": "ms"}, f)
        return path

    def summary(self) -> dict:
        """Per-name {count, total_ms, mean_ms} over host and GPU spans."""
        agg: dict = {}
        for ev in self.chrome_events():
            if ev.get("ph") != "X":
                continue
            key = f'{ev.get("cat")}:{ev["name"]}'
            a = agg.setdefault(key, [0, 0.0])
            a[0] += 1
            a[1] += ev["dur"] / 1e3
        return {k: {"count": n, "total_ms": round(t, 3), "mean_ms": round(t / n, 4)} for k, (n, t) in agg.items()}

    def clear(self):
        self.events.clear()
        self._gpu.clear()


_tracer: Tracer | None = None


def get_tracer() -> Tracer | None:
    """The active tracer, or None (the hot path checks this once per frame)."""
    return _tracer


def tracing_enabled() -> bool:
    return _tracer is not None


def enable_tracing(path: str | None = None, capacity: int | None = None) -> Tracer:
    global _tracer
    if _tracer is None:
        cap = capacity or int(os.environ.get("AIKO_TRACE_EVENTS", "1000000"))
        _tracer = Tracer(path, cap)
        if path:
            atexit.register(_export_at_exit)
    elif path:
        _tracer.path = path
    return _tracer


def disable_tracing() -> Tracer | None:
    global _tracer
    t, _tracer = _tracer, None
    return t


def _export_at_exit():
    if _tracer is not None and _tracer.path:
        try:
            _tracer.export()
        except Exception:      # exit path: never raise
            pass


if os.environ.get("AIKO_TRACE"):
    enable_tracing(os.environ["AIKO_TRACE"])
