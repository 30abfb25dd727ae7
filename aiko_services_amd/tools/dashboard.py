"""aiko_dashboard: terminal UI over the registrar and the services' EC shares
(reference ``main/dashboard.py`` + ``dashboard_plugins.py``, asciimatics -> stdlib curses).

Pages: the live services table (ServicesCache) with the selected service's shared variables
(ECConsumer on its ``/control`` topic) underneath; service history; the selected process's log
(``{process}/0/log``).  Keys: Up/Down select service, Tab/Enter move between panes, ``e`` edit
the selected variable (publishes ``(update name value)``), ``L`` cycle the service log level,
``l`` log page, ``h`` history, ``K`` kill the selected (local) process, ``q`` quit.  GPU
services show their device, HBM frame-pool occupancy and frames/s when they share them.

Plugins (reference ``dashboard_plugins.py``): ``PLUGINS`` maps a service *name* or *protocol* to
a page function ``page(dashboard, details, width) -> [lines]``; ``p`` shows the selected
service's plugin page.  Built in: ``registrar`` (discovered services' topic paths) and
``gpu`` pages for services that share GPU telemetry.  ``register_plugin(key, page)`` adds more.

``--snapshot`` prints the services (and optionally one service's variables) once and exits —
the scriptable / testable mode.
"""
from __future__ import annotations

import argparse
import os
import signal
import threading
import time
from collections import deque

from ..control.share import ECConsumer, services_cache_create_singleton
from ..runtime.process import aiko
from ..runtime.service import ServiceTopicPath
from ..utils.sexpr import generate

__all__ = ["Dashboard", "PLUGINS", "format_services", "main", "register_plugin"]

LOG_LEVELS = ["DEBUG", "INFO", "WARNING", "ERROR"]
HISTORY_LIMIT = 32
LOG_RING = 128


def _field(details, i, key):
    return details[key] if isinstance(details, dict) else details[i]


def format_services(services, width=120):
    rows = ["Topic                          Name                 Protocol                    Transport Owner    Tags"]
    for d in services:
        tp = ServiceTopicPath.parse(_field(d, 0, "topic_path"))
        topic = tp.terse if tp else str(_field(d, 0, "topic_path"))
        protocol = str(_field(d, 2, "protocol")).rsplit("/", 1)[-1]
        tags = _field(d, 5, "tags")
        tags = " ".join(tags) if isinstance(tags, list) else str(tags)
        rows.append(f"{topic:30.30} {str(_field(d, 1, 'name')):20.20} {protocol:27.27} "
                    f"{str(_field(d, 3, 'transport')):9.9} {str(_field(d, 4, 'owner')):8.8} {tags}"[:width])
    return rows


def registrar_page(dashboard, details, width=120):
    """Reference ``RegistrarFrame``: the registrar's view of every discovered service."""
    rows = ["Registrar: Discovered Services topic paths"]
    for d in dashboard.services():
        tp = ServiceTopicPath.parse(_field(d, 0, "topic_path"))
        rows.append(f"{str(tp) if tp else _field(d, 0, 'topic_path'):40.40} {str(_field(d, 1, 'name')):20.20} "
                    f"{str(_field(d, 4, 'owner')):10.10} {str(_field(d, 2, 'protocol'))}"[:width])
    return rows


GPU_KEYS = ("gpu", "device", "gpu_fps", "hbm", "rccl", "latency")


def gpu_page(dashboard, details, width=120):
    """GPU element telemetry from the selected service's share (device, HBM, RCCL, latency)."""
    rows = [f"GPU telemetry: {_field(details, 1, 'name')}"]
    for k, v in dashboard.flat_variables():
        if any(g in k for g in GPU_KEYS):
            rows.append(f"  {k:40.40} {v}"[:width])
    return rows


PLUGINS = {"registrar": registrar_page}


def register_plugin(key, page):
    """Add a plugin page for services whose name or protocol is ``key``."""
    PLUGINS[key] = page


def find_plugin(details):
    name = str(_field(details, 1, "name"))
    protocol = str(_field(details, 2, "protocol"))
    for key in (name, protocol, protocol.rsplit("/", 1)[-1].split(":")[0]):
        if key in PLUGINS:
            return PLUGINS[key]
    return None


class LogLevelPopupMenu:
    """Log-level chooser for the selected service (reference ``dashboard.py:670-714``): a small
    window listing the levels with the current one highlighted; up/down or a digit picks, enter
    applies — the choice is published as ``(update log_level LEVEL)`` on the service's
    ``/control`` topic, exactly like an edited variable."""

    def __init__(self, dashboard, levels=None):
        self.dashboard = dashboard
        self.levels = list(levels or LOG_LEVELS)
        current = str(dashboard.variables.get("log_level", "INFO")).upper()
        self.index = self.levels.index(current) if current in self.levels else 0

    def key(self, ch) -> str | None:
        """Feed one key: returns the chosen level on enter/digit, "" on cancel, None to go on."""
        if ch in (27, ord("q")):
            return ""
        if ord("1") <= ch < ord("1") + len(self.levels):
            self.index = ch - ord("1")
            return self.apply()
        if ch in (258, ord("j")):                     # curses.KEY_DOWN
            self.index = (self.index + 1) % len(self.levels)
        elif ch in (259, ord("k")):                   # curses.KEY_UP
            self.index = (self.index - 1) % len(self.levels)
        elif ch in (10, 13):
            return self.apply()
        return None

    def apply(self) -> str:
        level = self.levels[self.index]
        self.dashboard.edit_variable("log_level", level)
        return level

    def lines(self) -> list[str]:
        return [f"{'>' if i == self.index else ' '} {i + 1} {lv}" for i, lv in enumerate(self.levels)]

    def run(self, scr):
        import curses
        h, w = scr.getmaxyx()
        bw, bh = 18, len(self.levels) + 2
        win = curses.newwin(bh, bw, max(0, (h - bh) // 2), max(0, (w - bw) // 2))
        win.keypad(True)
        while True:
            win.erase()
            win.box()
            win.addstr(0, 2, " log level ")
            for i, line in enumerate(self.lines()):
                win.addstr(1 + i, 1, line[: bw - 2], curses.A_REVERSE if i == self.index else 0)
            win.refresh()
            out = self.key(win.getch())
            if out is not None:
                return out


class Dashboard:
    def __init__(self, history_limit=HISTORY_LIMIT):
        self.cache = services_cache_create_singleton(aiko.process, True, history_limit)
        self.selected = 0
        self.consumer = None
        self.variables: dict = {}
        self.selected_topic = None
        self.log_topic = None
        self.log: deque = deque(maxlen=LOG_RING)
        self.lock = threading.Lock()
        self.page = "services"
        self.focus = "services"
        self.var_index = 0
        self.status = ""

    # ---- data ------------------------------------------------------------------------------
    def services(self):
        return list(self.cache.get_services())

    def select(self, details):
        topic_path = _field(details, 0, "topic_path")
        if topic_path == self.selected_topic:
            return
        if self.consumer is not None:
            self.consumer.terminate()
            self.consumer = None
        self.variables = {}
        self.selected_topic = topic_path
        tags = _field(details, 5, "tags")
        if "ec=true" in (tags if isinstance(tags, list) else str(tags).split()):
            self.consumer = ECConsumer(aiko.process, 0, self.variables, f"{topic_path}/control")
        self._follow_log(topic_path)

    def _follow_log(self, topic_path):
        tp = ServiceTopicPath.parse(topic_path)
        new = f"{tp.topic_path_process}/0/log" if tp else None
        if new == self.log_topic:
            return
        if self.log_topic:
            aiko.process.remove_message_handler(self._log_handler, self.log_topic)
        self.log.clear()
        self.log_topic = new
        if new:
            aiko.process.add_message_handler(self._log_handler, new)

    def _log_handler(self, _aiko, topic, payload):
        with self.lock:
            self.log.append(str(payload))

    def edit_variable(self, name, value):
        if self.selected_topic:
            aiko.message.publish(f"{self.selected_topic}/control", generate("update", [name, value]))

    def cycle_log_level(self):
        current = str(self.variables.get("log_level", "INFO")).upper()
        nxt = LOG_LEVELS[(LOG_LEVELS.index(current) + 1) % len(LOG_LEVELS)] if current in LOG_LEVELS else "INFO"
        self.edit_variable("log_level", nxt)
        return nxt

    def kill_selected(self):
        tp = ServiceTopicPath.parse(self.selected_topic or "")
        if tp is None:
            return "no service selected"
        from ..utils.configuration import get_hostname
        if tp.hostname != get_hostname():
            return "can only kill local processes"
        try:
            os.kill(int(tp.process_id), signal.SIGKILL)
            return f"killed {tp.process_id}"
        except (OSError, ValueError) as exc:
            return str(exc)

    def flat_variables(self):
        out = []
        for k, v in sorted(self.variables.items()):
            if isinstance(v, dict):
                out.extend((f"{k}.{sk}", sv) for sk, sv in sorted(v.items()))
            else:
                out.append((k, v))
        return out

    def plugin_lines(self, width=120):
        services = self.services()
        if not services or self.selected >= len(services):
            return ["no service selected"]
        details = services[self.selected]
        page = find_plugin(details)
        if page is None and any(any(g in k for g in GPU_KEYS) for k, _ in self.flat_variables()):
            page = gpu_page
        if page is None:
            return [f"no plugin for {_field(details, 1, 'name')}"]
        return page(self, details, width)

    # ---- curses UI -------------------------------------------------------------------------
    def run_curses(self):
        import curses
        curses.wrapper(self._main)

    def _main(self, scr):
        import curses
        curses.curs_set(0)
        scr.timeout(250)
        while True:
            self._draw(scr)
            ch = scr.getch()
            if ch == -1:
                continue
            if ch in (ord("q"), 27):
                return
            services = self.services()
            if ch == curses.KEY_DOWN:
                if self.focus == "services":
                    self.selected = min(self.selected + 1, max(0, len(services) - 1))
                else:
                    self.var_index = min(self.var_index + 1, max(0, len(self.flat_variables()) - 1))
            elif ch == curses.KEY_UP:
                if self.focus == "services":
                    self.selected = max(0, self.selected - 1)
                else:
                    self.var_index = max(0, self.var_index - 1)
            elif ch in (9, 10, 13):
                self.focus = "variables" if self.focus == "services" else "services"
            elif ch == ord("l"):
                self.page = "log" if self.page != "log" else "services"
            elif ch == ord("h"):
                self.page = "history" if self.page != "history" else "services"
            elif ch == ord("p"):
                self.page = "plugin" if self.page != "plugin" else "services"
            elif ch == ord("L"):
                self.status = f"log_level -> {self.cycle_log_level()}"
            elif ch == ord("v"):
                chosen = LogLevelPopupMenu(self).run(scr)
                self.status = f"log_level -> {chosen}" if chosen else "log level unchanged"
            elif ch == ord("K"):
                self.status = self.kill_selected()
            elif ch == ord("e") and self.focus == "variables":
                vars_ = self.flat_variables()
                if vars_:
                    name = vars_[self.var_index][0]
                    value = self._prompt(scr, f"{name} = ")
                    if value is not None:
                        self.edit_variable(name, value)
                        self.status = f"update {name} {value}"
            if services and self.selected < len(services):
                from ..runtime import event
                event.call_soon(self.select, services[self.selected])

    def _prompt(self, scr, text):
        import curses
        h, w = scr.getmaxyx()
        curses.echo()
        scr.timeout(-1)
        scr.addstr(h - 1, 0, text[: w - 1])
        scr.clrtoeol()
        try:
            value = scr.getstr(h - 1, len(text), 200).decode()
        except Exception:
            value = None
        curses.noecho()
        scr.timeout(250)
        return value or None

    def _draw(self, scr):
        scr.erase()
        h, w = scr.getmaxyx()
        title = f" aiko dashboard (MI355X)  state={self.cache.get_state()}  {aiko.topic_path_process} "
        scr.addstr(0, 0, title[: w - 1])
        if self.page == "log":
            with self.lock:
                lines = list(self.log)[-(h - 3):]
            scr.addstr(1, 0, f"log: {self.log_topic}"[: w - 1])
            for i, line in enumerate(lines):
                scr.addstr(2 + i, 0, line[: w - 1])
        elif self.page == "plugin":
            rows = self.plugin_lines(w - 1)
            for i, row in enumerate(rows[: h - 2]):
                scr.addstr(1 + i, 0, row[: w - 1])
        elif self.page == "history":
            rows = format_services(list(self.cache.get_history()), w - 1)
            for i, row in enumerate(rows[: h - 2]):
                scr.addstr(1 + i, 0, row[: w - 1])
        else:
            rows = format_services(self.services(), w - 1)
            top = max(3, h // 2)
            for i, row in enumerate(rows[:top]):
                attr = 0
                if i - 1 == self.selected and self.focus == "services":
                    import curses
                    attr = curses.A_REVERSE
                scr.addstr(1 + i, 0, row[: w - 1], attr)
            scr.addstr(top + 1, 0, "-" * (w - 1))
            for i, (k, v) in enumerate(self.flat_variables()[: h - top - 4]):
                import curses
                attr = curses.A_REVERSE if (self.focus == "variables" and i == self.var_index) else 0
                scr.addstr(top + 2 + i, 0, f"{k:40.40} {v}"[: w - 1], attr)
        scr.addstr(h - 1, 0, (f"{self.status}  " + "q quit  arrows select  tab pane  e edit  v level menu  L next level  "
                              "l log  h history  p plugin  K kill")[: w - 1])
        scr.refresh()


def main(argv=None):
    ap = argparse.ArgumentParser(description="aiko dashboard")
    ap.add_argument("--history_limit", "-hl", type=int, default=HISTORY_LIMIT)
    ap.add_argument("--plugin", "-p", action="append", default=[],
                    help="module (or path/file.py) whose PLUGINS dict adds plugin pages (repeatable)")
    ap.add_argument("--snapshot", action="store_true", help="print services once and exit")
    ap.add_argument("--service", default=None, help="(snapshot) also print this service's variables")
    ap.add_argument("--timeout", type=float, default=5.0)
    a = ap.parse_args(argv)
    for module in a.plugin:
        from ..utils.misc import load_module
        PLUGINS.update(getattr(load_module(module), "PLUGINS", {}))
    dash = Dashboard(a.history_limit)
    if not a.snapshot:
        dash.run_curses()
        aiko.process.terminate()
        return
    if not dash.cache.wait_ready(a.timeout):
        print(f"registrar not ready (state={dash.cache.get_state()})")
    services = dash.services()
    for row in format_services(services):
        print(row)
    if a.service:
        from ..runtime import event
        for d in services:
            if a.service in (_field(d, 1, "name"), _field(d, 0, "topic_path")):
                event.call_soon(dash.select, d).result(5)
                deadline = time.time() + a.timeout
                while (dash.consumer is None or dash.consumer.cache_state != "ready") and time.time() < deadline:
                    time.sleep(0.05)
                for k, v in dash.flat_variables():
                    print(f"  {k} = {v}")
    aiko.process.terminate()


if __name__ == "__main__":
    main()
