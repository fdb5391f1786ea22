"""Lightweight Prometheus-text metrics (served on the REST port at /monitoring/prometheus/metrics).

Request count and latency histograms per RPC method and status code, batch
size histogram, queue depth and per-device busy time.  (The reference has no
metrics — SURVEY.md §5 — this is the server-side observability plan.)
"""
from __future__ import annotations

import bisect
import threading
import time
from collections import defaultdict
from typing import Dict, List, Tuple

LATENCY_BUCKETS = [1e-4, 2.5e-4, 5e-4, 1e-3, 2.5e-3, 5e-3, 1e-2, 2.5e-2, 5e-2, 0.1, 0.25, 0.5, 1, 2.5, 5, 10]
BATCH_BUCKETS = [1, 2, 4, 8, 16, 32, 64, 128, 256, 512]


class Histogram:
    def __init__(self, buckets):
        self.buckets = list(buckets)
        self.counts = [0] * (len(self.buckets) + 1)
        self.sum = 0.0
        self.n = 0

    def observe(self, v: float):
        self.counts[bisect.bisect_left(self.buckets, v)] += 1
        self.sum += v
        self.n += 1

    def quantile(self, q: float) -> float:
        if self.n == 0:
            return 0.0
        target = q * self.n
        acc = 0
        for i, c in enumerate(self.counts):
            acc += c
            if acc >= target:
                return self.buckets[i] if i < len(self.buckets) else float("inf")
        return float("inf")


class Metrics:
    def __init__(self):
        self._lock = threading.Lock()
        self.rpc_count: Dict[Tuple[str, int], int] = defaultdict(int)
        self.rpc_latency: Dict[str, Histogram] = {}
        self.batch_size = Histogram(BATCH_BUCKETS)
        self.batch_latency = Histogram(LATENCY_BUCKETS)
        self.queue_depth: Dict[str, int] = defaultdict(int)
        self.device_busy_s: Dict[str, float] = defaultdict(float)
        self.started = time.time()
        # extra exporters (e.g. the native transport's C++ counters): () -> [lines]
        self.collectors: List = []

    def observe_rpc(self, method: str, code: int, seconds: float):
        with self._lock:
            self.rpc_count[(method, code)] += 1
            h = self.rpc_latency.get(method)
            if h is None:
                h = self.rpc_latency[method] = Histogram(LATENCY_BUCKETS)
            h.observe(seconds)

    def observe_batch(self, size: int, seconds: float, device: str = ""):
        with self._lock:
            self.batch_size.observe(size)
            self.batch_latency.observe(seconds)
            if device:
                self.device_busy_s[device] += seconds

    def set_queue_depth(self, key: str, depth: int):
        with self._lock:
            self.queue_depth[key] = depth

    def render(self) -> str:
        out: List[str] = []
        with self._lock:
            out.append("# TYPE tfserve_request_count counter")
            for (m, c), n in sorted(self.rpc_count.items()):
                out.append(f'tfserve_request_count{{method="{m}",code="{c}"}} {n}')
            out.append("# TYPE tfserve_request_latency_seconds histogram")
            for m, h in sorted(self.rpc_latency.items()):
                out += _hist_lines("tfserve_request_latency_seconds", f'method="{m}"', h)
            out.append("# TYPE tfserve_batch_size histogram")
            out += _hist_lines("tfserve_batch_size", "", self.batch_size)
            out.append("# TYPE tfserve_batch_latency_seconds histogram")
            out += _hist_lines("tfserve_batch_latency_seconds", "", self.batch_latency)
            out.append("# TYPE tfserve_queue_depth gauge")
            for k, v in sorted(self.queue_depth.items()):
                out.append(f'tfserve_queue_depth{{queue="{k}"}} {v}')
            out.append("# TYPE tfserve_device_busy_seconds counter")
            for k, v in sorted(self.device_busy_s.items()):
                out.append(f'tfserve_device_busy_seconds{{device="{k}"}} {v:.6f}')
            out.append(f"tfserve_uptime_seconds {time.time() - self.started:.3f}")
            collectors = list(self.collectors)
        for c in collectors:
            try:
                out.extend(c())
            except Exception:       # a broken exporter must not break /metrics
                pass
        return "\n".join(out) + "\n"


def _hist_lines(name, labels, h: Histogram):
    sep = "," if labels else ""
    lines, acc = [], 0
    for b, c in zip(h.buckets + [float("inf")], h.counts):
        acc += c
        le = "+Inf" if b == float("inf") else repr(b)
        lines.append(f'{name}_bucket{{{labels}{sep}le="{le}"}} {acc}')
    lines.append(f"{name}_sum{{{labels}}} {h.sum:.6f}" if labels else f"{name}_sum {h.sum:.6f}")
    lines.append(f"{name}_count{{{labels}}} {h.n}" if labels else f"{name}_count {h.n}")
    return lines
