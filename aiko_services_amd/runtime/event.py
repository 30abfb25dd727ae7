"""Event engine: timers, typed queue, actor mailboxes and flat-out handlers on ONE loop thread.

Same public functions as the reference (``main/event.py:72-79``) — ``add_{flatout,mailbox,
queue,timer}_handler``, ``remove_*``, ``loop``, ``mailbox_put``, ``queue_put``, ``terminate`` —
but a different engine:

* wakeup-driven: producers (network threads, frame generators, other actors) signal a
  condition variable; the loop sleeps exactly until the next timer is due or work arrives.
  There is no fixed 10 ms tick and no "one queued message per iteration" throttle, which
  is what capped the reference at ~100 msgs/s per process;
* timers live in a heap keyed by due time (O(log n) add/remove instead of a linked list),
  identified by handler with duplicate-safe removal;
* priority is per mailbox (an actor's ``control`` mailbox), not "the first mailbox ever
  registered in the process"; a non-priority drain yields as soon as any priority mailbox
  has work;
* the clock is injectable (:class:`EventEngine` ``clock=``) so lease/timer logic is testable
  with virtual time.
"""
from __future__ import annotations

import heapq
import itertools
import threading
import time
from collections import OrderedDict, deque

__all__ = [
    "EventEngine", "Mailbox", "engine", "set_engine",
    "add_flatout_handler", "add_mailbox_handler", "add_queue_handler", "add_timer_handler",
    "loop", "mailbox_put", "queue_put",
    "remove_flatout_handler", "remove_mailbox_handler", "remove_queue_handler",
    "remove_timer_handler", "terminate", "is_running", "wakeup", "call_soon", "call_on_loop",
]

MAILBOX_INCREMENT_WARNING = 4


class Mailbox:
    __slots__ = ("handler", "name", "priority", "queue", "high_water_mark",
                 "increment_warning", "last_warned_increment", "put_count")

    def __init__(self, handler, name, priority=False, increment_warning=MAILBOX_INCREMENT_WARNING):
        self.handler = handler
        self.name = name
        self.priority = priority
        self.queue: deque = deque()
        self.high_water_mark = 0
        self.increment_warning = increment_warning
        self.last_warned_increment = 0
        self.put_count = 0

    @property
    def size(self):
        return len(self.queue)

    def put(self, item):
        self.queue.append(item)
        self.put_count += 1
        n = len(self.queue)
        if n > self.high_water_mark:
            self.high_water_mark = n
        if n >= self.last_warned_increment + self.increment_warning:
            self.last_warned_increment += self.increment_warning


class _Timer:
    __slots__ = ("handler", "period", "due", "seq", "cancelled")

    def __init__(self, handler, period, due, seq):
        self.handler = handler
        self.period = period
        self.due = due
        self.seq = seq
        self.cancelled = False

    def __lt__(self, other):
        return (self.due, self.seq) < (other.due, other.seq)


class EventEngine:
    def __init__(self, clock=time.time):
        self.clock = clock
        self._cv = threading.Condition(threading.Lock())
        self._timers: list = []                # heap of _Timer
        self._timers_by_handler: dict = {}     # handler -> [_Timer]
        self._seq = itertools.count()
        self._queue: deque = deque()
        self._queue_handlers: dict = {}
        self._mailboxes: "OrderedDict[str, Mailbox]" = OrderedDict()
        self._flatout: list = []
        self._handler_count = 0
        self._enabled = False
        self._running = False
        self._pending = False                  # work signalled since last drain
        self.loop_thread: threading.Thread | None = None
        self.stats = {"iterations": 0, "queue_items": 0, "mailbox_items": 0, "timer_calls": 0}

    # ---- registration ---------------------------------------------------------------------
    def add_flatout_handler(self, handler):
        with self._cv:
            self._flatout.append(handler)
            self._handler_count += 1
            self._cv.notify()

    def remove_flatout_handler(self, handler):
        with self._cv:
            if handler in self._flatout:
                self._flatout.remove(handler)
                self._handler_count -= 1

    def add_mailbox_handler(self, handler, name, increment_warning=MAILBOX_INCREMENT_WARNING,
                            priority=None):
        with self._cv:
            if name in self._mailboxes:
                raise RuntimeError(f"Mailbox {name}: Already exists")
            if priority is None:
                priority = name.endswith("/control")
            self._mailboxes[name] = Mailbox(handler, name, priority, increment_warning)
            self._handler_count += 1

    def remove_mailbox_handler(self, handler, name):
        with self._cv:
            if self._mailboxes.pop(name, None) is not None:
                self._handler_count -= 1

    def mailbox_put(self, name, item):
        with self._cv:
            mailbox = self._mailboxes.get(name)
            if mailbox is None:
                raise RuntimeError(f"Mailbox {name}: Not found")
            mailbox.put((item, self.clock()))
            self._pending = True
            self._cv.notify()

    def mailbox(self, name) -> Mailbox | None:
        return self._mailboxes.get(name)

    def add_queue_handler(self, handler, item_types=("default",)):
        with self._cv:
            for t in item_types:
                self._queue_handlers.setdefault(t, []).append(handler)
                self._handler_count += 1

    def remove_queue_handler(self, handler, item_types=("default",)):
        with self._cv:
            for t in item_types:
                handlers = self._queue_handlers.get(t)
                if handlers and handler in handlers:
                    handlers.remove(handler)
                    self._handler_count -= 1
                if handlers is not None and not handlers:
                    del self._queue_handlers[t]

    def queue_put(self, item, item_type="default"):
        with self._cv:
            self._queue.append((item, item_type))
            self._pending = True
            self._cv.notify()

    def add_timer_handler(self, handler, time_period, immediate=False):
        with self._cv:
            now = self.clock()
            t = _Timer(handler, float(time_period), now if immediate else now + time_period,
                       next(self._seq))
            heapq.heappush(self._timers, t)
            self._timers_by_handler.setdefault(handler, []).append(t)
            self._handler_count += 1
            self._cv.notify()

    def remove_timer_handler(self, handler):
        """Remove the most recently added timer for ``handler`` (no-op if absent)."""
        with self._cv:
            timers = self._timers_by_handler.get(handler)
            if not timers:
                return False
            t = timers.pop()
            if not timers:
                del self._timers_by_handler[handler]
            t.cancelled = True
            self._handler_count -= 1
            return True

    def has_timer(self, handler) -> bool:
        return bool(self._timers_by_handler.get(handler))

    def call_soon(self, fn, *args, **kwargs):
        """Run ``fn`` on the loop thread; returns a ``concurrent.futures.Future``."""
        import concurrent.futures
        fut = concurrent.futures.Future()

        def runner(_item, _type):
            if not fut.set_running_or_notify_cancel():
                return
            try:
                fut.set_result(fn(*args, **kwargs))
            except BaseException as exc:  # delivered to the caller
                fut.set_exception(exc)

        with self._cv:
            self._queue.append(((runner,), "__call__"))
            self._pending = True
            self._cv.notify()
        return fut

    def wakeup(self):
        with self._cv:
            self._pending = True
            self._cv.notify()

    # ---- the loop ---------------------------------------------------------------------------
    def _next_due(self):
        while self._timers and self._timers[0].cancelled:
            heapq.heappop(self._timers)
        return self._timers[0].due if self._timers else None

    def _run_due_timers(self):
        now = self.clock()
        while True:
            with self._cv:
                due = self._next_due()
                if due is None or due > now:
                    return
                t = heapq.heappop(self._timers)
                # reschedule before calling: the handler may remove itself
                t.due = max(t.due + t.period, now) if t.period > 0 else now
                t.seq = next(self._seq)
                heapq.heappush(self._timers, t)
            self.stats["timer_calls"] += 1
            t.handler()
            if t.period <= 0:
                return  # zero-period timers run at most once per iteration

    def _drain_queue(self):
        while True:
            with self._cv:
                if not self._queue:
                    return
                item, item_type = self._queue.popleft()
                handlers = list(self._queue_handlers.get(item_type, ())) if item_type != "__call__" \
                    else [item[0]]
            self.stats["queue_items"] += 1
            for h in handlers:
                h(item, item_type)

    def _priority_pending(self):
        for mb in self._mailboxes.values():
            if mb.priority and mb.queue:
                return True
        return False

    def _drain_mailboxes(self):
        progressed = True
        while progressed:
            progressed = False
            # priority mailboxes first, fully
            for mb in list(self._mailboxes.values()):
                if mb.priority:
                    while mb.queue:
                        item, t = mb.queue.popleft()
                        self.stats["mailbox_items"] += 1
                        mb.handler(mb.name, item, t)
                        progressed = True
            for mb in list(self._mailboxes.values()):
                if mb.priority:
                    continue
                while mb.queue:
                    item, t = mb.queue.popleft()
                    self.stats["mailbox_items"] += 1
                    mb.handler(mb.name, item, t)
                    progressed = True
                    if self._priority_pending():
                        break
                if self._priority_pending():
                    break

    def _has_work(self):
        if self._queue:
            return True
        for mb in self._mailboxes.values():
            if mb.queue:
                return True
        return False

    def loop(self, loop_when_no_handlers=False):
        with self._cv:
            if self._running:
                return
            self._running = True
            self._enabled = True
            self.loop_thread = threading.current_thread()
            # timers restart relative to loop start (reference EventList.reset())
            now = self.clock()
            for t in self._timers:
                if not t.cancelled and t.due < now and t.period > 0:
                    pass
        try:
            while self._enabled and (loop_when_no_handlers or self._handler_count > 0):
                self.stats["iterations"] += 1
                self._run_due_timers()
                self._drain_queue()
                self._drain_mailboxes()
                if self._flatout:
                    for h in list(self._flatout):
                        h()
                    continue
                with self._cv:
                    if not self._enabled:
                        break
                    if self._has_work() or self._pending:
                        self._pending = False
                        continue
                    due = self._next_due()
                    timeout = None if due is None else max(0.0, due - self.clock())
                    if timeout is None and not loop_when_no_handlers and self._handler_count == 0:
                        break
                    if timeout is None or timeout > 0:
                        self._cv.wait(timeout if timeout is not None else 1.0)
                    self._pending = False
        except KeyboardInterrupt:
            raise SystemExit("KeyboardInterrupt: abort !")
        finally:
            with self._cv:
                self._running = False
                self.loop_thread = None

    def run_once(self):
        """One non-blocking pass (used by tests driving a virtual clock)."""
        self._run_due_timers()
        self._drain_queue()
        self._drain_mailboxes()
        for h in list(self._flatout):
            h()

    def terminate(self):
        with self._cv:
            self._enabled = False
            self._cv.notify_all()

    def is_running(self):
        return self._running

    def reset(self):
        """Drop every handler (tests / process re-initialisation)."""
        with self._cv:
            self._timers.clear()
            self._timers_by_handler.clear()
            self._queue.clear()
            self._queue_handlers.clear()
            self._mailboxes.clear()
            self._flatout.clear()
            self._handler_count = 0


engine = EventEngine()


def set_engine(new_engine: EventEngine) -> EventEngine:
    global engine
    old = engine
    engine = new_engine
    return old


# ---- module-level API (reference names) ------------------------------------------------------

def add_flatout_handler(handler):
    engine.add_flatout_handler(handler)


def remove_flatout_handler(handler):
    engine.remove_flatout_handler(handler)


def add_mailbox_handler(mailbox_handler, mailbox_name, mailbox_increment_warning=MAILBOX_INCREMENT_WARNING,
                        priority=None):
    engine.add_mailbox_handler(mailbox_handler, mailbox_name, mailbox_increment_warning, priority)


def remove_mailbox_handler(mailbox_handler, mailbox_name):
    engine.remove_mailbox_handler(mailbox_handler, mailbox_name)


def mailbox_put(mailbox_name, item):
    engine.mailbox_put(mailbox_name, item)


def add_queue_handler(queue_handler, item_types=("default",)):
    engine.add_queue_handler(queue_handler, item_types)


def remove_queue_handler(queue_handler, item_types=("default",)):
    engine.remove_queue_handler(queue_handler, item_types)


def queue_put(item, item_type="default"):
    engine.queue_put(item, item_type)


def add_timer_handler(handler, time_period, immediate=False):
    engine.add_timer_handler(handler, time_period, immediate)


def remove_timer_handler(handler):
    return engine.remove_timer_handler(handler)


def loop(loop_when_no_handlers=False):
    engine.loop(loop_when_no_handlers)


def terminate():
    engine.terminate()


def is_running():
    return engine.is_running()


def wakeup():
    engine.wakeup()


def call_soon(fn, *args, **kwargs):
    return engine.call_soon(fn, *args, **kwargs)


def call_on_loop(fn, *args, timeout=10.0, **kwargs):
    """Run ``fn`` on the event loop thread and wait for its result (or run inline when the
    caller already is the loop thread or no loop is running)."""
    if not engine.is_running() or threading.current_thread() is engine.loop_thread:
        return fn(*args, **kwargs)
    return engine.call_soon(fn, *args, **kwargs).result(timeout)


def __getattr__(name):
    # reference compatibility: ``event.event_loop_running``
    if name == "event_loop_running":
        return engine.is_running()
    raise AttributeError(name)
