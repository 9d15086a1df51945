"""Per-rank heartbeat + hang watchdog (reference: workers block in NCCL until the 1800 s
process-group timeout, ``training.py:249-256,285``, with only ``NCCL_DEBUG=INFO`` logs to go on,
``deploy/pytorchjob.yaml:51-64``).

Every rank records where it is — step, phase, last gradient bucket launched — as ONE line:

* in a file ``$SFTAMD_HEARTBEAT_DIR/rank<r>.hb`` (replaced atomically at every beat), which the launcher
  (``launch.py``) watches: a rank whose file stops changing for ``--hang-timeout`` seconds is a hang, and the
  launcher prints every rank's last line before tearing the group down;
* on stderr, throttled (``SFTAMD_HEARTBEAT_STDERR_S``, default 30 s, plus the first beat of every step until
  step 3), so a job log shows the last known position of each rank even when nothing else is printed;
* an in-process watchdog thread (``SFTAMD_HANG_TIMEOUT_S`` > 0, or ``Heartbeat(hang_timeout_s=...)``): when no
  beat arrives for that long — a collective that never completes, a peer that died without the launcher noticing
  (e.g. under an external ``torchrun``) — it prints the last heartbeat and exits the process with code 124 instead
  of waiting for the process-group timeout. ``deadline_s`` bounds the whole run the same way.

Phases that legitimately run long without beats — checkpoint I/O (rank 0 writes while the others wait in a
barrier), checkpoint loading, the first step (GEMM tuning, extension warm-up) — run inside ``hold(phase)``,
which allows them the slow-phase limit (``SFTAMD_SLOW_PHASE_TIMEOUT_S``, default max(4 x hang timeout, 1800 s))
instead of the hang timeout (the limit goes into every beat record as ``limit_s``, which the launcher's watchdog
honours too); ``pause()`` / ``resume()`` switch the hang check off outside the training loop (before ``train()``
and after it returns), where nothing beats at all — except inside a ``hold``. The deadline always applies.

A beat is a few microseconds of host work (no device sync); with no directory, no stderr cadence and no
watchdog configured, ``beat`` is a no-op.
"""
from __future__ import annotations

import contextlib
import json
import os
import sys
import threading
import time
from typing import Optional

EXIT_HANG = 124


def _fmt(rec: dict) -> str:
    return json.dumps(rec, separators=(",", ":"), sort_keys=False)


class Heartbeat:
    def __init__(self, rank: int, directory: Optional[str] = None, stderr_every_s: Optional[float] = None,
                 hang_timeout_s: Optional[float] = None, deadline_s: Optional[float] = None, info=None):
        self.rank = rank
        self.dir = directory if directory is not None else os.environ.get("SFTAMD_HEARTBEAT_DIR") or None
        if stderr_every_s is None:
            stderr_every_s = float(os.environ.get("SFTAMD_HEARTBEAT_STDERR_S", "30"))
        self.stderr_every = stderr_every_s
        if hang_timeout_s is None:
            hang_timeout_s = float(os.environ.get("SFTAMD_HANG_TIMEOUT_S", "0") or 0)
        self.hang_timeout = hang_timeout_s
        slow = float(os.environ.get("SFTAMD_SLOW_PHASE_TIMEOUT_S", "0") or 0)
        self.slow_timeout = slow if slow > 0 else max(4.0 * hang_timeout_s, 1800.0)
        self._limit = hang_timeout_s  # the in-process hang limit in force (raised inside hold())
        self._hold_limit = 0.0  # > 0 inside hold(): the slow-phase limit, written into every record for launch.py
        self._paused = False
        if deadline_s is None:
            deadline_s = float(os.environ.get("SFTAMD_RUN_DEADLINE_S", "0") or 0) or None
        self.deadline = deadline_s
        self.info = info  # optional callable -> dict merged into every record (e.g. the DDP engine's bucket)
        self.t0 = time.time()
        self.last = {"rank": rank, "step": 0, "phase": "start", "t": 0.0}
        self._last_beat = time.monotonic()
        self._last_err = 0.0
        self._err_steps = set()
        self._stop = threading.Event()
        self.path = None
        if self.dir:
            os.makedirs(self.dir, exist_ok=True)
            self.path = os.path.join(self.dir, f"rank{rank}.hb")
        self.enabled = bool(self.path or self.stderr_every > 0 or self.hang_timeout > 0 or self.deadline)
        self._thread = None
        if self.hang_timeout > 0 or self.deadline:
            self._thread = threading.Thread(target=self._watch, name=f"sftamd-watchdog-{rank}", daemon=True)
            self._thread.start()
        self.beat(0, "start")

    # ------------------------------------------------------------------ beats
    def beat(self, step: Optional[int] = None, phase: str = "", **extra):
        if not self.enabled:
            return
        now = time.time()
        rec = {"rank": self.rank, "step": self.last["step"] if step is None else int(step), "phase": phase,
               "t": round(now - self.t0, 3)}
        if self.info is not None:
            try:
                rec.update(self.info())
            except Exception:
                pass
        rec.update(extra)
        if self._paused:
            rec["paused"] = True  # launch.py skips the hang check of a paused rank
        elif self._hold_limit > 0:
            # ... and applies a hold's longer limit — written whether or not THIS process runs its own watchdog: a
            # launcher-only watchdog (launch.py --hang-timeout, children without SFTAMD_HANG_TIMEOUT_S) reads it too
            rec["limit_s"] = self._hold_limit
        self.last = rec
        self._last_beat = time.monotonic()
        line = _fmt(rec)
        if self.path:
            tmp = f"{self.path}.tmp"
            try:
                with open(tmp, "w") as f:
                    f.write(line + "\n")
                os.replace(tmp, self.path)
            except OSError:
                pass
        s = rec["step"]
        if self.stderr_every > 0 and (now - self._last_err >= self.stderr_every or
                                      (s <= 3 and s not in self._err_steps)):
            self._last_err = now
            self._err_steps.add(s)
            print(f"[heartbeat] {line}", file=sys.stderr, flush=True)

    @contextlib.contextmanager
    def hold(self, phase: str, timeout_s: Optional[float] = None, step: Optional[int] = None):
        """A phase allowed ``timeout_s`` (default: the slow-phase limit) without beats; beats on entry and exit.
        A hold also lifts ``pause()`` for its duration: a held phase outside the training loop (the final save and
        its barrier) keeps the slow-phase limit instead of no hang check at all."""
        prev, prev_hold, prev_paused = self._limit, self._hold_limit, self._paused
        self._hold_limit = max(self.hang_timeout, timeout_s or self.slow_timeout)
        if self.hang_timeout > 0:
            self._limit = self._hold_limit
        self._paused = False
        self.beat(step, phase)
        try:
            yield
        finally:
            self._limit, self._hold_limit = prev, prev_hold
            self._last_beat = time.monotonic()
            self._paused = prev_paused
            self.beat(step, f"{phase}_done")

    def pause(self):
        """No hang check until ``resume()`` (the deadline still applies)."""
        self._paused = True
        self.beat(None, "idle")

    def resume(self):
        self._last_beat = time.monotonic()
        self._paused = False
        self.beat(None, "resume")

    # ------------------------------------------------------------------ watchdog
    def _watch(self):
        while not self._stop.wait(1.0):
            idle = time.monotonic() - self._last_beat
            over = self.deadline and time.time() - self.t0 > self.deadline
            limit = self._limit
            if (limit > 0 and not self._paused and idle > limit) or over:
                why = (f"deadline of {self.deadline:.0f} s exceeded" if over else
                       f"no progress for {idle:.0f} s (hang limit {limit:.0f} s)")
                print(f"[watchdog] rank {self.rank}: {why}; last heartbeat {_fmt(self.last)}", file=sys.stderr,
                      flush=True)
                os._exit(EXIT_HANG)

    def close(self):
        self._stop.set()


def read_heartbeats(directory: str, n: int):
    """Last heartbeat line of ranks 0..n-1 (None where a rank never wrote one) and each file's age in seconds."""
    out = []
    now = time.time()
    for r in range(n):
        p = os.path.join(directory, f"rank{r}.hb")
        try:
            with open(p) as f:
                line = f.read().strip()
            out.append((r, line, now - os.path.getmtime(p)))
        except OSError:
            out.append((r, None, None))
    return out


_GLOBAL: Optional[Heartbeat] = None


def get() -> Optional[Heartbeat]:
    return _GLOBAL


def install(hb: Heartbeat) -> Heartbeat:
    global _GLOBAL
    _GLOBAL = hb
    return hb
