"""Collective watchdog: a host thread that turns a hung step into a gang restart.

Reference behaviour: "ModelCheckpoint callback is not provided. Workers will need to
restart training if any fails" (README.md:400) -- TF has no way out of a collective whose
peer died.  Here (SURVEY.md §5 failure detection):

* ``fit`` arms the watchdog for the whole training loop; after enqueuing each chunk of
  steps it hands the watchdog a device event recorded behind that chunk
  (:meth:`Watchdog.beat_when_done`), and the watchdog thread beats when the event
  COMPLETES -- so a beat means the chunk's device work (kernels, RCCL / xGMI exchanges)
  finished, not merely that the host enqueued it, and a wedged collective is detected one
  deadline after the last completed chunk;
* a daemon thread checks the age of the last beat; past the deadline it logs which phase
  was stuck, aborts the registered communicators (``ncclCommAbort`` wakes a device-side
  RCCL wait, the peer kernel's bounded waits expire on their own) and ends the process with
  exit status :data:`EXIT_CODE` -- never ``exec``, never a retry in place;
* the launcher sees the non-zero exit, kills the gang and restarts it
  (``launch_script(max_restarts=...)``), and ``BackupAndRestore`` resumes from the last
  epoch backup.

``DAMD_WATCHDOG_S``: deadline in seconds (default 300 when the job has more than one
worker, 0 = off; single-worker jobs have no collective to hang and default to off).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, List, Optional

from . import env
from . import logging as dlog

EXIT_CODE = 75  # EX_TEMPFAIL: "try again" -- the launcher's cue for a gang restart


class Watchdog:
    def __init__(self, deadline_s: float, on_expire: Optional[Callable[[str], None]] = None, poll_s: float = 0.5):
        self.deadline_s = float(deadline_s)
        self.poll_s = min(poll_s, max(0.05, self.deadline_s / 10))
        self._on_expire = on_expire
        self._aborts: List[Callable[[], None]] = []
        self._last = time.monotonic()
        self._phase = "start"
        self._armed = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._pending: List[tuple] = []  # (event, phase) in enqueue order
        self._lock = threading.Lock()
        self.fired = False

    # --- control ---------------------------------------------------------------------
    def add_abort(self, fn: Callable[[], None]) -> None:
        """Called (in registration order) when the deadline expires, before the exit."""
        self._aborts.append(fn)

    def arm(self, phase: str = "train") -> "Watchdog":
        self._last = time.monotonic()
        self._phase = phase
        self._armed = True
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, name="damd-watchdog", daemon=True)
            self._thread.start()
        return self

    def beat(self, phase: Optional[str] = None) -> None:
        self._last = time.monotonic()
        if phase is not None:
            self._phase = phase

    def beat_when_done(self, event, phase: str) -> None:
        """Beat when ``event`` (anything with ``query() -> bool``, e.g. a torch.cuda.Event
        recorded behind a chunk of device work) completes; events complete in order."""
        with self._lock:
            self._pending.append((event, phase))

    def _poll_events(self) -> None:
        with self._lock:
            while self._pending:
                ev, phase = self._pending[0]
                try:
                    done = bool(ev.query())
                except Exception:  # pragma: no cover - a destroyed / failed event counts as done
                    done = True
                if not done:
                    break
                self._pending.pop(0)
                self._last = time.monotonic()
                self._phase = phase

    def disarm(self) -> None:
        self._armed = False

    def close(self) -> None:
        self._armed = False
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2.0)
            self._thread = None

    def __enter__(self):
        return self.arm()

    def __exit__(self, *exc):
        self.close()
        return False

    # --- thread ----------------------------------------------------------------------
    def _run(self) -> None:
        while not self._stop.wait(self.poll_s):
            if not self._armed:
                continue
            self._poll_events()
            age = time.monotonic() - self._last
            if age > self.deadline_s:
                self._expire(age)
                return

    def _expire(self, age: float) -> None:
        self.fired = True
        msg = (f"collective watchdog: no progress for {age:.1f}s (deadline {self.deadline_s:.1f}s) "
               f"in phase '{self._phase}'; aborting communicators and exiting with status {EXIT_CODE} "
               "for a gang restart")
        dlog.error(msg)
        for fn in self._aborts:
            try:
                fn()
            except Exception as e:  # pragma: no cover - best effort on the way out
                dlog.error("watchdog abort hook failed: %s", e)
        if self._on_expire is not None:
            self._on_expire(msg)
            return
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(EXIT_CODE)


def deadline_for(world_size: int) -> float:
    default = 300.0 if world_size > 1 else 0.0
    return env.get_float("DAMD_WATCHDOG_S", default)


def for_strategy(strategy) -> Optional[Watchdog]:
    """A watchdog for a training loop under ``strategy`` (None when disabled), with the
    strategy's communicator abort registered."""
    d = deadline_for(strategy.num_replicas_in_sync)
    if d <= 0:
        return None
    wd = Watchdog(d)
    comm = strategy.communicator
    nat = getattr(comm, "native", None)
    if nat is not None and hasattr(nat, "abort"):
        wd.add_abort(nat.abort)
    return wd
