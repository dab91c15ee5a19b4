"""Engine liveness: "is the engine making progress on the work it has?"

The reference's replicas are judged by the ALB health check (``/health`` every 10 s, unhealthy after
10 failures, sd21-weighted-routing-ing.yaml:9-14) and the K8s probes, which only prove that the HTTP
server answers -- a replica stuck in a hung kernel stays "healthy".  Here every engine loop reports
progress (a finished job / engine step) and whether work is pending; ``/health`` turns 503 once work has
been pending for longer than ``SHAI_HANG_TIMEOUT_S`` without progress, so the router drains the replica and
the supervisor's watchdog (``supervisor.health.GPUHealthMonitor.check_workers``) kills and restarts it.
"""
from __future__ import annotations

import os
import threading
import time

DEFAULT_HANG_TIMEOUT_S = float(os.environ.get("SHAI_HANG_TIMEOUT_S", "180"))


class Liveness:
    def __init__(self, hang_timeout_s: float = DEFAULT_HANG_TIMEOUT_S, clock=time.monotonic):
        self.hang_timeout_s = hang_timeout_s
        self.clock = clock
        self._lock = threading.Lock()
        self.last_progress = clock()
        self.pending_since = None
        self.progress_count = 0

    def work_pending(self) -> None:
        """Work was queued (or is in flight)."""
        with self._lock:
            if self.pending_since is None:
                self.pending_since = self.clock()

    def progress(self, still_pending: bool) -> None:
        """One unit of work completed (a job, an engine step)."""
        with self._lock:
            now = self.clock()
            self.last_progress = now
            self.progress_count += 1
            self.pending_since = now if still_pending else None

    def stalled_for(self) -> float:
        """Seconds that pending work has waited without any progress (0 when idle)."""
        with self._lock:
            if self.pending_since is None:
                return 0.0
            return max(0.0, self.clock() - max(self.pending_since, self.last_progress))

    @property
    def healthy(self) -> bool:
        return self.stalled_for() <= self.hang_timeout_s

    def snapshot(self) -> dict:
        return {"stalled_s": round(self.stalled_for(), 3), "hang_timeout_s": self.hang_timeout_s,
                "progress_count": self.progress_count, "pending": self.pending_since is not None}


_REGISTRY: list = []
_BROKEN: "str | None" = None


def mark_broken(reason: str) -> None:
    """A fault this process cannot recover from in place (a TP peer collective timed out, a TP rank died):
    ``/health`` answers 503 from now on, so the router drains the replica and the supervisor restarts the
    whole group.  The first reason is kept."""
    global _BROKEN
    if _BROKEN is None:
        _BROKEN = str(reason)
        try:
            from .logging import get_logger
            get_logger("liveness").error("process marked broken", extra={"event": "broken", "detail": _BROKEN})
        except Exception:  # noqa: BLE001 -- never let reporting mask the fault
            pass


def broken() -> "str | None":
    """The reason this process was marked broken, or None."""
    return _BROKEN


def _reset_broken_for_tests() -> None:
    global _BROKEN
    _BROKEN = None


def register(live: "Liveness") -> "Liveness":
    """Make ``live`` part of this process's ``/health`` verdict (every engine loop registers one)."""
    _REGISTRY.append(live)
    return live


def worst() -> "Liveness | None":
    """The registered engine that has been stalled longest (None when none is registered)."""
    return max(_REGISTRY, key=lambda l: l.stalled_for() - l.hang_timeout_s, default=None)
