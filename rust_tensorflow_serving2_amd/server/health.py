"""Replica health: detect a servable whose device keeps failing and reload it.

SURVEY.md §5 "Failure detection / elastic recovery": the reference has none
(errors bubble up as ``Box<dyn Error>``, ``src/lib.rs:11``); TF Serving marks a
failed load ``END`` with an error status (``get_model_status.proto:50-60``).
Serving on GPUs adds a failure mode the load path never sees: a servable that
loaded fine starts failing every batch (a HIP error, a wedged stream, a
corrupted graph).  Policy:

* Every executed batch reports success or failure per (model, version):
  the Python path through :meth:`HealthMonitor.record` (called by the serving
  core around each run), the C++ fast-path lanes through their endpoint
  counters (``failed`` / ``consecutive_failed`` in ``endpoint_stats``) which a
  watcher thread polls.  Client errors (bad shapes, unknown aliases) are not
  device failures and are not counted.
* ``threshold`` consecutive failures with no success in between mark the
  version unhealthy: the manager unloads it (draining nothing — its batches are
  failing anyway) and loads it again from disk (:meth:`ModelManager.recover`).
  Other versions and models keep serving throughout.
* After ``max_recoveries`` reloads of one version it is quarantined: state
  ``END`` with ``UNAVAILABLE`` and the last failure in its status, until a
  config reload asks for it again.

The one-process-per-GPU topology (``parallel/replicas.py``) makes this
per-GPU: each replica process runs its own monitor over its own device.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Dict, Iterable, List, Optional, Tuple

from . import errors as E

log = logging.getLogger("tfserve.health")

# codes that say "the server could not run the batch", as opposed to "the
# request was wrong" (INVALID_ARGUMENT, NOT_FOUND, FAILED_PRECONDITION, ...)
DEVICE_FAILURE_CODES = (E.INTERNAL, E.UNKNOWN, E.DATA_LOSS)
STICKY_EXIT = 75      # exit status of a replica that gave its poisoned GPU context up
_STICKY_WORDS = ("illegal address", "illegal memory", "hardware exception", "device not responding",
                 "timed out (device")


def is_sticky(why: str) -> bool:
    w = why.lower()
    return any(k in w for k in _STICKY_WORDS)


_DEVICE_WORDS = ("hip", "cuda", "gpu", "device", "hsa", "illegal memory", "illegal address")


def is_device_failure(exc: BaseException) -> bool:
    """True for errors raised by the GPU runtime (HIP / torch device errors)
    or by fault injection; host-side bugs (an IndexError in the reference
    interpreter, ...) and client errors are not device failures.  A wrapper
    error carries the verdict of what it wraps in ``device_failure``."""
    tag = getattr(exc, "device_failure", None)
    if tag is not None:
        return bool(tag)
    if isinstance(exc, E.ServingError):
        return exc.code in DEVICE_FAILURE_CODES
    from ..utils.faults import InjectedFault
    if isinstance(exc, InjectedFault):
        return True
    if isinstance(exc, RuntimeError):
        msg = str(exc).lower()
        return any(w in msg for w in _DEVICE_WORDS)
    return False


class HealthMonitor:
    def __init__(self, manager, threshold: int = 8, max_recoveries: int = 3, poll_s: float = 0.25, metrics=None,
                 clean_batches: int = 1000, clean_seconds: float = 600.0):
        self.manager = manager
        self.threshold = max(1, int(threshold))
        self.max_recoveries = int(max_recoveries)
        self.poll_s = poll_s
        # a recovered version that then serves `clean_batches` good batches, or
        # stays up `clean_seconds` without tripping, starts from zero again:
        # transient faults days apart must not add up to a quarantine
        self.clean_batches = int(clean_batches)
        self.clean_seconds = float(clean_seconds)
        self._lock = threading.Lock()
        self._consec: Dict[Tuple[str, int], int] = {}
        self._native_seen: Dict[Tuple[str, int, str], int] = {}
        self._native_batches: Dict[Tuple[str, int, str], int] = {}
        self._good: Dict[Tuple[str, int], int] = {}          # good batches since the last recovery
        self._recovered_at: Dict[Tuple[str, int], float] = {}
        self.failures: Dict[Tuple[str, int], int] = {}
        # reloads in the current window (decides quarantine; forgiven after a
        # clean run) and in total (the exported counter, never reset)
        self.recoveries: Dict[Tuple[str, int], int] = {}
        self.recoveries_total: Dict[Tuple[str, int], int] = {}
        hooks = getattr(manager, "config_listeners", None)
        if hooks is not None:        # an explicit config reload lifts quarantine: start over
            hooks.append(self.reset_model)
        self._sources: List[Callable[[], Iterable[Tuple[str, int, str, int, int]]]] = []
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        if metrics is not None:
            metrics.collectors.append(self.prometheus_lines)

    # --------------------------------------------------------------- reports
    def reset_model(self, name: str) -> None:
        """Forget the recovery history of every version of ``name``."""
        with self._lock:
            for d in (self.recoveries, self._good, self._recovered_at, self._consec):
                for k in [k for k in d if k[0] == name]:
                    del d[k]

    def _good_batches(self, key: Tuple[str, int], n: int) -> None:
        """(lock held) ``n`` more good batches of ``key``."""
        if not self.recoveries.get(key):
            return
        g = self._good.get(key, 0) + n
        self._good[key] = g
        if g >= self.clean_batches:
            self._forgive(key)

    def _forgive(self, key: Tuple[str, int]) -> None:
        log.info("model %s version %d healthy again: recovery count reset", *key)
        self.recoveries.pop(key, None)
        self._good.pop(key, None)
        self._recovered_at.pop(key, None)

    def record(self, name: str, version: int, ok: bool, why: str = "") -> None:
        key = (name, int(version))
        with self._lock:
            if ok:
                self._consec[key] = 0
                self._good_batches(key, 1)
                return
            self.failures[key] = self.failures.get(key, 0) + 1
            n = self._consec.get(key, 0) + 1
            self._consec[key] = n
            trip = n >= self.threshold
            if trip:
                self._consec[key] = 0
        if trip:
            if is_sticky(why):
                self._sticky(name, int(version), f"{n} consecutive failed batches; last: {why}")
            else:
                self._trip(name, int(version), f"{n} consecutive failed batches; last: {why}")

    def add_source(self, fn: Callable[[], Iterable[Tuple[str, int, str, int, int]]]) -> None:
        """``fn()`` yields ``(model, version, signature, failed_total, consecutive_failed)``
        for native executors (polled; the C++ lanes report no per-batch callback)."""
        self._sources.append(fn)
        if self._thread is None:
            self._thread = threading.Thread(target=self._poll, name="tfs-health", daemon=True)
            self._thread.start()

    def _poll(self) -> None:
        while not self._stop.wait(self.poll_s):
            for src in list(self._sources):
                try:
                    rows = list(src())
                except Exception:       # a source being torn down
                    continue
                for row in rows:
                    name, version, sig, failed, consec = row[:5]
                    batches = row[5] if len(row) > 5 else None
                    dead_lanes = row[6] if len(row) > 6 else 0
                    if dead_lanes:
                        self._sticky(name, int(version), f"{dead_lanes} GPU lane(s) timed out (device hang)")
                    k = (name, int(version), sig)
                    with self._lock:
                        new = failed - self._native_seen.get(k, 0)
                        self._native_seen[k] = failed
                        if new > 0:
                            self.failures[(name, int(version))] = self.failures.get((name, int(version)), 0) + new
                        if batches is not None:
                            prev = self._native_batches.get(k)
                            self._native_batches[k] = batches
                            good = batches - (prev if prev is not None and prev <= batches else batches) - max(new, 0)
                            if good > 0 and consec == 0:
                                self._good_batches((name, int(version)), good)
                    if consec >= self.threshold:
                        self._trip(name, int(version), f"{consec} consecutive failed batches on the GPU fast path")

    def _sticky(self, name: str, version: int, why: str) -> None:
        """A failure an in-process reload cannot fix (a hung queue, an illegal
        address: the HIP context is poisoned).  Under the replica supervisor
        (parallel/replicas.py, TFSERVE_SUPERVISED=1) the process exits so a
        fresh one takes the GPU; unsupervised, fall back to a reload."""
        if os.environ.get("TFSERVE_SUPERVISED") == "1":
            log.critical("model %s version %d: %s; exiting so the supervisor restarts this replica",
                         name, version, why)
            logging.shutdown()
            os._exit(STICKY_EXIT)
        self._trip(name, version, why)

    def _trip(self, name: str, version: int, why: str) -> None:
        key = (name, version)
        with self._lock:
            t = self._recovered_at.get(key)
            if t is not None and time.monotonic() - t >= self.clean_seconds:
                self._forgive(key)         # up long enough since the last reload
            n = self.recoveries.get(key, 0)
        quarantine = n >= self.max_recoveries
        # only a version that is AVAILABLE is taken down; repeated trips while
        # it is already unloading / reloading (the poller still sees the old
        # endpoint's counters) are no-ops and are not counted
        if not self.manager.recover(name, version, why, quarantine=quarantine):
            return
        if not quarantine:
            with self._lock:
                self.recoveries[key] = self.recoveries.get(key, 0) + 1
                self.recoveries_total[key] = self.recoveries_total.get(key, 0) + 1
                self._good[key] = 0
                self._recovered_at[key] = time.monotonic()
        log.error("model %s version %d unhealthy (%s); %s", name, version, why,
                  "quarantined" if quarantine else f"reloading (recovery {n + 1}/{self.max_recoveries})")

    # --------------------------------------------------------------- exports
    def prometheus_lines(self) -> List[str]:
        with self._lock:
            f = dict(self.failures)
            r = dict(self.recoveries_total)
        out = ["# TYPE tfserve_batch_failures_total counter"]
        out += [f'tfserve_batch_failures_total{{model="{m}",version="{v}"}} {n}' for (m, v), n in sorted(f.items())]
        out.append("# TYPE tfserve_servable_recoveries_total counter")
        out += [f'tfserve_servable_recoveries_total{{model="{m}",version="{v}"}} {n}'
                for (m, v), n in sorted(r.items())]
        return out

    def close(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
