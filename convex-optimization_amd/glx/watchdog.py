"""Per-rank watchdog for multi-rank runs (round 6).

A collective that never completes (a rank that died, a peer stuck on another call, an RCCL
transport fault) blocks every other rank inside that collective: on the device (RCCL kernels
spinning on a peer) or on the host (the host transport's gloo call). Without a watchdog the run
is killed at the launcher's time limit and says nothing. With it, each rank that passes its
deadline writes one diagnostic block to stderr and exits non-zero:

    glx watchdog: rank R of N: <what> passed its deadline of D s (elapsed E s)
      <probe>: <record>          # e.g. the session's iterations, the collectives issued
      ... every thread's Python stack (faulthandler) ...

and leaves through ``os._exit`` (never an exec: the process has initialised the GPU). The probes
are callables registered by the caller (``glx.Session.progress``, ``glx.dist.Comm.progress``);
they read thread-safe records from libglx (glx_session_progress / glx_comm_progress), so the
watchdog can run while the main thread is blocked inside the library. ctypes releases the GIL
around every libglx call, so the watchdog thread is never starved by a blocked solver call.
"""
from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Callable, Dict, Optional

EXIT_CODE = 3


class Watchdog:
    def __init__(self, deadline_s: float, what: str, rank: int = 0, world: int = 1,
                 exit_code: int = EXIT_CODE, stream=None, poll_s: float = 0.5):
        self.deadline_s = float(deadline_s)
        self.what = what
        self.rank, self.world = rank, world
        self.exit_code = exit_code
        self.stream = stream if stream is not None else sys.stderr
        self.poll_s = poll_s
        self._probes: Dict[str, Callable[[], object]] = {}
        self._t0 = time.monotonic()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.phase = "start"

    def probe(self, name: str, fn: Optional[Callable[[], object]]) -> None:
        """Register (fn) or drop (None) a progress probe printed when the deadline passes."""
        if fn is None:
            self._probes.pop(name, None)
        else:
            self._probes[name] = fn

    def start(self) -> "Watchdog":
        if self.deadline_s > 0 and self._thread is None:
            self._t0 = time.monotonic()
            self._thread = threading.Thread(target=self._run, name="glx-watchdog", daemon=True)
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
            self._thread = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def report(self, elapsed: float) -> str:
        lines = ["glx watchdog: rank %d of %d: %s passed its deadline of %.0f s (elapsed %.1f s, "
                 "phase %s)" % (self.rank, self.world, self.what, self.deadline_s, elapsed, self.phase)]
        for name, fn in list(self._probes.items()):
            try:
                rec = fn()
            except Exception as e:   # a probe must never keep the diagnostic from printing
                rec = "probe failed: %r" % (e,)
            lines.append("  %s: %s" % (name, rec))
        return "\n".join(lines)

    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            elapsed = time.monotonic() - self._t0
            if elapsed < self.deadline_s:
                continue
            try:
                self.stream.write(self.report(elapsed) + "\n")
                self.stream.write("  thread stacks:\n")
                self.stream.flush()
                faulthandler.dump_traceback(file=self.stream, all_threads=True)
                self.stream.flush()
            finally:
                os._exit(self.exit_code)
