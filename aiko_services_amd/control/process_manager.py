"""ProcessManager: spawn and supervise child processes (reference ``main/process_manager.py``).

``create(id, command, arguments, env=None, gpu=None)`` starts a child (a module name is
resolved to its file with ``importlib.util.find_spec``; ``.py``/``.sh`` run directly); a
monitor thread polls every 0.2 s and reports exits through ``process_exit_handler(id,
data)``.  MI355X addition: ``gpu=<index>`` pins the child to one GPU by setting
``HIP_VISIBLE_DEVICES`` (one worker process per GPU), and children keep
``HSA_ENABLE_IPC_MODE_LEGACY=0`` for dmabuf IPC.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import threading
import time
from subprocess import Popen

__all__ = ["ProcessManager", "PROCESS_POLL_TIME"]

PROCESS_POLL_TIME = 0.2


class ProcessManager:
    def __init__(self, process_exit_handler=None):
        self.process_exit_handler = process_exit_handler
        self.processes: dict = {}
        self.thread = None
        self._lock = threading.Lock()

    def __str__(self):
        return "\n".join(f"{id}: {d['process'].pid} {d['command_line'][0]}"
                         for id, d in self.processes.items())

    def create(self, id, command, arguments=None, env=None, gpu=None, cwd=None):
        command_line = [command]
        ext = os.path.splitext(command)[-1]
        if ext not in (".py", ".sh") and "/" not in command:
            try:
                spec = importlib.util.find_spec(command)
            except (ImportError, ValueError):
                spec = None
            if spec and spec.origin:
                command_line = [sys.executable, spec.origin]
        elif ext == ".py":
            command_line = [sys.executable, command]
        if arguments:
            command_line.extend(str(a) for a in arguments)
        child_env = dict(os.environ if env is None else env)
        child_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if gpu is not None:
            child_env["HIP_VISIBLE_DEVICES"] = str(gpu)
        process = Popen(command_line, bufsize=0, shell=False, env=child_env, cwd=cwd)
        with self._lock:
            self.processes[id] = {"command_line": command_line, "process": process,
                                  "return_code": None, "gpu": gpu}
            if self.thread is None or not self.thread.is_alive():
                self.thread = threading.Thread(target=self.run, daemon=True, name="process-manager")
                self.thread.start()
        return process

    def delete(self, id, terminate=True, kill=False):
        with self._lock:
            data = self.processes.pop(id, None)
        if data is None:
            return
        process = data["process"]
        if terminate and process.poll() is None:
            process.terminate()
        if kill and process.poll() is None:
            process.kill()
        if self.process_exit_handler:
            self.process_exit_handler(id, data)

    def wait(self, id, timeout=None):
        data = self.processes.get(id)
        return None if data is None else data["process"].wait(timeout)

    def run(self):
        while True:
            with self._lock:
                items = list(self.processes.items())
            if not items:
                return
            for id, data in items:
                rc = data["process"].poll()
                if rc is not None:
                    data["return_code"] = rc
                    self.delete(id, terminate=False, kill=False)
            time.sleep(PROCESS_POLL_TIME)

    def terminate_all(self, kill_after=2.0):
        with self._lock:
            ids = list(self.processes)
        for id in ids:
            self.delete(id, terminate=True)


def process_exit_handler_default(id, process_data):
    details = ""
    if process_data:
        details = f": {process_data['command_line'][0]} status: {process_data['return_code']}"
    print(f"Exit process {id}" + details)


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="ProcessManager example")
    ap.add_argument("--example", default=None, help="shell | python")
    a = ap.parse_args(argv)
    pm = ProcessManager(process_exit_handler_default)
    if a.example == "shell":
        pm.create("A", "/bin/sh", ["-c", "echo Start A; sleep 1; echo Stop A"])
        pm.create("B", "/bin/sh", ["-c", "echo Start B; sleep 2; echo Stop B"])
        time.sleep(3)
    elif a.example == "python":
        pm.create("P", sys.executable, ["-c", "print('hello from child')"])
        time.sleep(1)


if __name__ == "__main__":
    main()
