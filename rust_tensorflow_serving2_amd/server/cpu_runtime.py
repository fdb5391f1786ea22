"""Batched CPU execution behind the native fast path (BASELINE config 1:
half_plus_two on CPU).

Without this, a CPU servable answered every Predict in Python: decode, run,
encode, one GIL-bound round trip per request (2,092 RPC/s at 13.8 ms p50 in
round 1).  ``CpuRunner`` exposes the same lane interface as ``GpuRunner``
(``gpu_runtime.py``): the C++ endpoint decodes requests and copies their rows
into a lane's host buffers, a Python lane thread runs the compiled CPU program
once per BATCH on views of those buffers and writes the outputs back in place,
and the C++ side encodes every response.  Python work is per batch, not per
request, and the request / response bytes never enter Python.
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..utils import tensors as T
from .gpu_runtime import buckets_for


class CpuRunner:
    """Runner for a CPU servable whose inputs are batched (leading -1, static
    rest, numeric): ``run`` for the Python path, lanes for the fast path."""

    def __init__(self, base, lanes: int):
        self._base = base                       # servable.Runner (the compiled program)
        self.servable = base.servable
        self.in_specs = base.in_specs
        self.out_specs = base.out_specs
        self.program = base.program
        opts = self.servable.options
        self.buckets = buckets_for(opts.max_batch_size, opts.allowed_batch_sizes)
        self.n_lanes = max(1, lanes)
        self._host: List[Optional[Tuple[List[np.ndarray], List[np.ndarray]]]] = [None] * self.n_lanes
        self._lock = threading.Lock()

    # ------------------------------------------------------------ Python path
    def run(self, inputs: Sequence) -> List:
        return self._base.run(inputs)

    # ------------------------------------------------------------ fast path lanes
    def fast_lanes(self) -> List[int]:
        return list(range(self.n_lanes))

    def claim(self, lane_idx: int) -> None:
        pass

    def native_lane_spec(self, lane_idx: int):
        return None                             # lanes are Python threads (no device graphs)

    def _alloc(self, lane_idx: int):
        bmax = self.buckets[-1]
        ins = [np.zeros([bmax] + list(s.shape[1:]), dtype=T.np_dtype(s.dtype)) for s in self.in_specs]
        # output rows: shapes / dtypes of one probe batch (the signature may leave them open)
        probe = self.program.run([torch.from_numpy(a[:1]) for a in ins])
        outs = []
        for s, v in zip(self.out_specs, probe):
            v = v.detach().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            want = T.np_dtype(s.dtype) if s.dtype != T.DT_STRING else v.dtype
            outs.append(np.zeros((bmax,) + tuple(v.shape[1:]), dtype=want))
        return ins, outs

    def lane_host_pointers(self, lane_idx: int) -> Tuple[List[int], List[int]]:
        with self._lock:
            if self._host[lane_idx] is None:
                self._host[lane_idx] = self._alloc(lane_idx)
            ins, outs = self._host[lane_idx]
        return [a.ctypes.data for a in ins], [a.ctypes.data for a in outs]

    def run_lane(self, lane_idx: int, n: int) -> None:
        ins, outs = self._host[lane_idx]
        res = self.program.run([torch.from_numpy(a[:n]) for a in ins])
        for dst, v in zip(outs, res):
            v = v.detach().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
            if v.shape[0] != n or v.shape[1:] != dst.shape[1:]:
                raise RuntimeError(f"output rows {v.shape} do not match the lane buffer {dst.shape}")
            dst[:n] = v


def batched(in_specs, out_specs) -> bool:
    """Every input and output has a leading batch dim and static numeric rows."""
    def ok(s):
        return (s.shape is not None and len(s.shape) >= 1 and s.shape[0] == -1 and
                all(d >= 0 for d in s.shape[1:]) and s.dtype != T.DT_STRING)
    return all(ok(s) for s in in_specs) and all(ok(s) for s in out_specs)
