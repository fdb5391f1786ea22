"""Dynamic batching for the general (non-fast-path) request path.

TF Serving's ``--enable_batching`` semantics (``BatchingParameters`` in
``protos/tf_serving.proto``; the reference only ever sends batch-1 requests,
``src/lib.rs:229``, so server-side batching is what turns its traffic into
GPU-sized work):

* requests for the same (servable, signature, input aliases, output aliases,
  per-example shapes/dtypes) share a queue; their tensors are concatenated
  along dim 0 into one batch of at most ``max_batch_size`` rows;
* a batch closes when full or ``batch_timeout_micros`` after its first task;
  closed batches run on ``num_batch_threads`` workers;
* the batch is padded up to the next ``allowed_batch_sizes`` entry (by
  repeating the first row, as TF does) -- on the GPU these are exactly the
  HIP-graph buckets, so a padded batch replays a captured graph;
* ``max_enqueued_batches`` bounds the queue: beyond it requests fail fast
  with UNAVAILABLE instead of queueing unbounded latency;
* a request larger than ``max_batch_size`` is rejected (INVALID_ARGUMENT),
  with ``pad_variable_length_inputs`` ragged non-batch dims are zero-padded
  to the batch maximum.

The native transport's Predict fast path does the same thing in C++
(``csrc/batcher.cpp``) without the GIL; this module serves everything else
(grpcio transport, REST, Classify/Regress, signatures the fast path does not
take).
"""
from __future__ import annotations

import logging
import threading
import time
from collections import deque
from typing import Deque, Dict, List, Optional, Sequence

import numpy as np

from ..utils import roctx
from . import errors as E

log = logging.getLogger("tfserve.batching")


def _iv(msg, field: str, default: int) -> int:
    if msg is not None and msg.HasField(field):
        return int(getattr(msg, field).value)
    return default


class _Task:
    __slots__ = ("inputs", "size", "event", "result", "error")

    def __init__(self, inputs: Dict[str, np.ndarray], size: int):
        self.inputs = inputs
        self.size = size
        self.event = threading.Event()
        self.result: Optional[Dict[str, np.ndarray]] = None
        self.error: Optional[BaseException] = None


class _Batch:
    __slots__ = ("tasks", "size", "opened", "closed")

    def __init__(self):
        self.tasks: List[_Task] = []
        self.size = 0
        self.opened = time.perf_counter()
        self.closed = False


class _Queue:
    def __init__(self, servable, sig_name: str, in_aliases, out_aliases):
        self.servable = servable
        self.sig_name = sig_name
        self.in_aliases = in_aliases
        self.out_aliases = out_aliases
        self.open: Optional[_Batch] = None
        self.ready: Deque[_Batch] = deque()


class BatchingSession:
    def __init__(self, params=None, metrics=None):
        self.max_batch_size = _iv(params, "max_batch_size", 32)
        self.batch_timeout_s = _iv(params, "batch_timeout_micros", 1000) / 1e6
        self.max_enqueued_batches = _iv(params, "max_enqueued_batches", 64)
        self.num_batch_threads = max(1, _iv(params, "num_batch_threads", 4))
        allowed = sorted(int(x) for x in params.allowed_batch_sizes) if params is not None else []
        if allowed and allowed[-1] != self.max_batch_size:
            raise E.invalid("allowed_batch_sizes: the last entry must equal max_batch_size "
                            f"({allowed[-1]} != {self.max_batch_size})")
        if any(b <= 0 for b in allowed) or len(set(allowed)) != len(allowed):
            raise E.invalid("allowed_batch_sizes must be positive and strictly increasing")
        self.allowed_batch_sizes = allowed or [b for b in (1, 2, 4, 8, 16, 32, 64, 128, 256)
                                               if b < self.max_batch_size] + [self.max_batch_size]
        self.pad_variable_length_inputs = bool(params.pad_variable_length_inputs) if params is not None else False
        self.metrics = metrics
        self._cv = threading.Condition()
        self._queues: Dict[tuple, _Queue] = {}
        self._stop = False
        self._threads = [threading.Thread(target=self._worker, name=f"tfs-batch-{i}", daemon=True)
                         for i in range(self.num_batch_threads)]
        for t in self._threads:
            t.start()

    @property
    def timeout_us(self) -> int:
        return int(round(self.batch_timeout_s * 1e6))

    # ------------------------------------------------------------ public
    def run(self, servable, sig_name: str, inputs: Dict[str, np.ndarray], out_aliases: Sequence[str]):
        arrs = {a: np.asarray(v) for a, v in inputs.items()}
        if not arrs or any(v.ndim == 0 for v in arrs.values()) or any(v.dtype == object for v in arrs.values()):
            return servable.run(sig_name, inputs, out_aliases)       # not batchable
        sizes = {v.shape[0] for v in arrs.values()}
        if len(sizes) != 1:
            raise E.invalid("Batching session Run() input tensors must have equal 0th-dimension size")
        n = sizes.pop()
        if n == 0:
            return servable.run(sig_name, inputs, out_aliases)
        if n > self.max_batch_size:
            raise E.invalid(f"Task size {n} is larger than maximum input batch size {self.max_batch_size}")
        in_aliases = tuple(sorted(arrs))
        if self.pad_variable_length_inputs:
            shape_key = tuple((a, arrs[a].dtype.str, arrs[a].ndim) for a in in_aliases)
        else:
            shape_key = tuple((a, arrs[a].dtype.str, arrs[a].shape[1:]) for a in in_aliases)
        key = (id(servable), sig_name, tuple(out_aliases), shape_key)
        task = _Task(arrs, n)
        with self._cv:
            if self._stop:
                raise E.unavailable("batching session is shutting down")
            q = self._queues.get(key)
            if q is None or q.servable is not servable:
                q = self._queues[key] = _Queue(servable, sig_name, in_aliases, tuple(out_aliases))
            b = q.open
            if b is not None and b.size + n > self.max_batch_size:
                self._close(q)
                b = None
            if b is None:
                if len(q.ready) >= self.max_enqueued_batches:
                    raise E.unavailable("The batch scheduling queue to which this session was assigned is full")
                b = q.open = _Batch()
            b.tasks.append(task)
            b.size += n
            if b.size >= self.max_batch_size:
                self._close(q)
            self._cv.notify_all()
        task.event.wait()
        if task.error is not None:
            raise task.error
        return task.result

    def stop(self):
        with self._cv:
            self._stop = True
            for q in self._queues.values():
                if q.open is not None:
                    self._close(q)
            self._cv.notify_all()
        for t in self._threads:
            t.join(timeout=10)

    def queue_depth(self) -> int:
        with self._cv:
            return sum(len(q.ready) + (q.open is not None) for q in self._queues.values())

    # ------------------------------------------------------------ internals
    def _close(self, q: _Queue):
        b = q.open
        q.open = None
        if b is not None and not b.closed:
            b.closed = True
            q.ready.append(b)

    def _next(self):
        """Pick the next runnable batch (holding ``_cv``); returns (queue, batch) or a wait time."""
        now = time.perf_counter()
        wait = None
        best = None
        for key, q in list(self._queues.items()):
            if q.open is not None and now - q.open.opened >= self.batch_timeout_s:
                self._close(q)
            if q.ready:
                b = q.ready[0]
                if best is None or b.opened < best[1].opened:
                    best = (q, b)
            elif q.open is not None:
                left = self.batch_timeout_s - (now - q.open.opened)
                wait = left if wait is None else min(wait, left)
            elif q.servable.bundle is None:        # unloaded servable: drop its idle queue
                del self._queues[key]
        if best is not None:
            best[0].ready.popleft()
            return best
        return wait

    def _worker(self):
        while True:
            with self._cv:
                while True:
                    nxt = self._next()
                    if isinstance(nxt, tuple):
                        break
                    if self._stop:
                        return
                    self._cv.wait(timeout=nxt if nxt is not None else 0.5)
                if self.metrics is not None:
                    self.metrics.set_queue_depth("batching", sum(len(q.ready) for q in self._queues.values()))
            q, b = nxt
            self._execute(q, b)

    def _padded(self, n: int) -> int:
        for s in self.allowed_batch_sizes:
            if s >= n:
                return s
        return n

    def _execute(self, q: _Queue, b: _Batch):
        t0 = time.perf_counter()
        try:
            total = b.size
            target = self._padded(total)
            feeds = {}
            for a in q.in_aliases:
                parts = [t.inputs[a] for t in b.tasks]
                if self.pad_variable_length_inputs:
                    parts = _pad_ragged(parts)
                x = parts[0] if len(parts) == 1 else np.concatenate(parts, axis=0)
                if target > total:
                    x = np.concatenate([x, np.repeat(x[:1], target - total, axis=0)], axis=0)
                feeds[a] = x
            fault = getattr(q.servable, "fault", None)
            if fault is not None:
                fault.check()
            with roctx.range(f"tfs.batch rows={target}") if roctx.enabled() else roctx.NULL:
                outs = q.servable.run(q.sig_name, feeds, list(q.out_aliases))
            off = 0
            for t in b.tasks:
                res = {}
                for a, v in outs.items():
                    if v.ndim == 0 or v.shape[0] != target:
                        raise E.internal("Batched output tensor's 0th dimension does not equal the sum of "
                                         "the 0th dimension sizes of the input tensors")
                    res[a] = v[off:off + t.size]
                t.result = res
                off += t.size
        except BaseException as e:     # every task of the batch gets the (same) error
            if isinstance(e, E.ServingError):
                err = e
            else:
                from .health import is_device_failure
                err = E.internal(f"{type(e).__name__}: {e}")
                err.device_failure = is_device_failure(e)     # host bugs are not device failures
            for t in b.tasks:
                t.error = err
        finally:
            if self.metrics is not None:
                self.metrics.observe_batch(b.size, time.perf_counter() - t0, q.servable.options.device)
            for t in b.tasks:
                t.event.set()


def _pad_ragged(parts: List[np.ndarray]) -> List[np.ndarray]:
    nd = parts[0].ndim
    mx = [max(p.shape[d] for p in parts) for d in range(1, nd)]
    out = []
    for p in parts:
        pad = [(0, 0)] + [(0, m - s) for m, s in zip(mx, p.shape[1:])]
        out.append(np.pad(p, pad) if any(w for _, w in pad) else p)
    return out
