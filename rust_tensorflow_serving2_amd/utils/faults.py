"""Fault injection for failure-detection tests (SURVEY.md §5 "Failure detection").

``TFSERVE_FAULT`` holds comma-separated ``key=value`` items; the C++ fast-path
lanes (``csrc/server.cpp``, class ``NativeLane``) parse the same spec:

* ``lane_every=N`` — every Nth batch fails (a transient device error);
* ``lane_after=N`` — every batch after the first N fails (a device that went
  bad: the replica health monitor must take the servable down and reload it).

Counts are per executor (a native lane, or the Python batch executor of one
servable), so a reloaded servable starts counting from zero again.
"""
from __future__ import annotations

import os
import threading
from typing import Dict, Optional


def parse(spec: Optional[str]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for item in (spec or "").split(","):
        k, sep, v = item.strip().partition("=")
        if sep and k in ("lane_every", "lane_after"):
            out[k] = int(v)
    return out


class FaultPoint:
    """Counts executions; :meth:`check` raises when the spec says this one fails."""

    def __init__(self, spec: Optional[str] = None):
        f = parse(os.environ.get("TFSERVE_FAULT") if spec is None else spec)
        self.every = f.get("lane_every", 0)
        self.after = f.get("lane_after", -1)
        self.enabled = self.every > 0 or self.after >= 0
        self._n = 0
        self._lock = threading.Lock()

    def check(self) -> None:
        if not self.enabled:
            return
        with self._lock:
            self._n += 1
            n = self._n
        if (self.every > 0 and n % self.every == 0) or (self.after >= 0 and n > self.after):
            raise InjectedFault("injected fault (TFSERVE_FAULT)")


class InjectedFault(RuntimeError):
    """Stands in for a HIP runtime error in tests."""
