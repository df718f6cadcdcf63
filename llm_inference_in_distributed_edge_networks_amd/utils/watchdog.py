"""Progress watchdog (the reference has no failure detection).

A daemon thread expects ``beat()`` at least every ``timeout_s`` seconds.  If progress stalls (a dead
pipeline peer, a hung collective, a kernel that never finishes) it dumps every thread's Python stack
to stderr and terminates the process with exit code 70, so ``torchrun`` tears the whole job down
instead of leaving ranks blocked forever.  The process-group timeout covers collectives; this covers
everything else.  Enable with ``EDGE_WATCHDOG_S=<seconds>`` or construct explicitly.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time


class Watchdog:
    def __init__(self, timeout_s: float, name: str = "edge", on_timeout=None):
        self.timeout_s = float(timeout_s)
        self.name = name
        self.on_timeout = on_timeout
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name=f"{name}-watchdog", daemon=True)
        self.fired = False

    def start(self) -> "Watchdog":
        self._thread.start()
        return self

    def beat(self) -> None:
        self._last = time.monotonic()

    def stop(self) -> None:
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(1.0, self.timeout_s / 4)):
            if time.monotonic() - self._last > self.timeout_s:
                self.fired = True
                print(f"[{self.name}] watchdog: no progress for {self.timeout_s:.0f}s, dumping stacks",
                      file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                if self.on_timeout is not None:
                    self.on_timeout()
                    return
                os._exit(70)

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


def from_env(name: str = "edge"):
    s = os.environ.get("EDGE_WATCHDOG_S")
    return Watchdog(float(s), name).start() if s else None
