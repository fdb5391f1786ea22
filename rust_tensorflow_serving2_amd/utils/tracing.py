"""Request / batch tracing (``--trace_dir``).

Two sources, one clock (CLOCK_MONOTONIC, microseconds):

* native GPU lanes record one span set per batch in C++
  (``Http2Server.drain_trace``): batch opened (first row reserved) -> closed
  and acquired by the lane -> GPU done -> responses posted;
* the Python core records one span per RPC it handles (slow path / other RPCs).

A background thread appends JSON lines to ``<trace_dir>/trace-<pid>.jsonl``;
``scripts/trace_to_chrome.py`` turns them into a chrome://tracing / Perfetto
timeline.  The reference has no tracing at all.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import List, Optional


def now_us() -> float:
    return time.monotonic() * 1e6


class Tracer:
    def __init__(self, trace_dir: str, flush_s: float = 1.0):
        os.makedirs(trace_dir, exist_ok=True)
        self.path = os.path.join(trace_dir, f"trace-{os.getpid()}.jsonl")
        self._f = open(self.path, "a", buffering=1 << 16)
        self._lock = threading.Lock()
        self._pending: List[dict] = []
        self._servers = []
        self._stop = threading.Event()
        self._flush_s = flush_s
        self._th = threading.Thread(target=self._loop, name="tfs-trace", daemon=True)
        self._th.start()

    def attach_native(self, srv) -> None:
        """Start collecting batch spans from a native Http2Server."""
        srv.set_tracing(True)
        self._servers.append(srv)

    def rpc(self, method: str, t0_us: float, t1_us: float, code: int) -> None:
        with self._lock:
            self._pending.append({"type": "rpc", "method": method, "start_us": t0_us, "end_us": t1_us, "code": code})

    def _collect(self) -> List[dict]:
        with self._lock:
            out, self._pending = self._pending, []
        for srv in self._servers:
            for ep, slot, rows, opened, acq, issued, done, posted in srv.drain_trace():
                out.append({"type": "batch", "endpoint": ep, "slot": slot, "rows": rows, "opened_us": opened,
                            "acquired_us": acq, "issued_us": issued, "done_us": done, "posted_us": posted})
        return out

    def flush(self) -> None:
        recs = self._collect()
        if recs:
            self._f.write("".join(json.dumps(r) + "\n" for r in recs))
            self._f.flush()

    def _loop(self):
        while not self._stop.wait(self._flush_s):
            self.flush()

    def close(self) -> None:
        self._stop.set()
        self._th.join(timeout=5)
        for srv in self._servers:
            try:
                srv.set_tracing(False)
            except Exception:
                pass
        self.flush()
        self._f.close()


def load(path: str) -> List[dict]:
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def to_chrome(records: List[dict]) -> dict:
    """chrome://tracing JSON: one track per (endpoint, slot) with queue / gpu /
    respond phases per batch, and one track per RPC method."""
    ev = []
    for r in records:
        if r["type"] == "batch":
            tid = f"endpoint {r['endpoint']} lane {r['slot']}"
            for name, a, b in (("batch forming", r["opened_us"], r["acquired_us"]),
                               ("H2D+graph+D2H", r["acquired_us"], r["done_us"]),
                               ("encode+post", r["done_us"], r["posted_us"])):
                ev.append({"name": name, "ph": "X", "pid": "gpu lanes", "tid": tid, "ts": a, "dur": max(0.0, b - a),
                           "args": {"rows": r["rows"]}})
        elif r["type"] == "rpc":
            ev.append({"name": r["method"].rsplit("/", 1)[-1], "ph": "X", "pid": "python core", "tid": r["method"],
                       "ts": r["start_us"], "dur": max(0.0, r["end_us"] - r["start_us"]), "args": {"code": r["code"]}})
    return {"traceEvents": ev, "displayTimeUnit": "ms"}
