"""GPU execution of a signature on one MI355X: fused HIP program + HIP graphs.

* The signature's Program is compiled with the fusion passes on ``cuda:N``:
  bf16 weights resident in HBM, fused conv/GEMM/attention kernels.
* Requests are padded up to a *batch bucket* (``allowed_batch_sizes``, else
  powers of two up to ``max_batch_size``).  Each bucket is warmed up eagerly
  once (kernel tile autotuning happens here), then captured into a HIP graph
  with static input/output buffers; serving a batch is one H2D copy into the
  static inputs, one ``graph.replay()``, one D2H copy of the outputs.
* ``lanes`` independent (stream, buffers, graphs) sets let the H2D copy and
  compute of consecutive batches overlap (one lane in flight per stream).
"""
from __future__ import annotations

import logging
import threading
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from ..graph.compiler import compile_program
from ..utils import tensors as T
from . import errors as E

log = logging.getLogger("tfserve.gpu")


def buckets_for(max_batch: int, allowed: Sequence[int] = ()) -> List[int]:
    if allowed:
        return sorted(set(int(a) for a in allowed))
    out, b = [], 1
    while b < max_batch:
        out.append(b)
        b *= 2
    out.append(max_batch)
    return sorted(set(out))


class _Lane:
    def __init__(self, device):
        self.stream = torch.cuda.Stream(device=device)
        self.lock = threading.Lock()
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.static_in: Dict[int, List[torch.Tensor]] = {}
        self.static_out: Dict[int, List[torch.Tensor]] = {}
        self.host_in: Dict[int, List[torch.Tensor]] = {}
        self.host_out: Dict[int, List[torch.Tensor]] = {}


class GpuRunner:
    def __init__(self, servable, in_specs, out_specs, lanes: int = 2):
        self.servable = servable
        self.in_specs = in_specs
        self.out_specs = out_specs
        self.device = servable.options.torch_device
        opts = servable.options
        g = servable.fresh_graph()
        with torch.cuda.device(self.device):
            self.program = compile_program(g, [s.name for s in in_specs], [s.name for s in out_specs],
                                           self.device, servable.passes(), opts.extra)
        self.batched = all(s.shape is not None and len(s.shape) >= 1 and s.shape[0] == -1 and
                           all(d >= 0 for d in s.shape[1:]) and s.dtype != T.DT_STRING for s in in_specs)
        self.use_graphs = opts.hip_graphs and self.batched
        self.buckets = buckets_for(opts.max_batch_size, opts.allowed_batch_sizes)
        self.lanes = [_Lane(self.device) for _ in range(max(1, lanes))]
        self._rr = 0
        self._rr_lock = threading.Lock()
        self._out_dt = [s.dtype for s in out_specs]

    # ------------------------------------------------------------ helpers
    def _to_device_dtype(self, spec, arr: np.ndarray) -> torch.Tensor:
        from .servable import _np_to_torch
        return _np_to_torch(arr, spec.dtype)

    def _finish(self, outs: List) -> List:
        res = []
        for v, dt in zip(outs, self._out_dt):
            if isinstance(v, torch.Tensor) and v.dtype == torch.bfloat16 and dt == T.DT_FLOAT:
                v = v.float()
            res.append(v)
        return res

    def _eager(self, feeds: List) -> List:
        with torch.cuda.device(self.device):
            dev_feeds = [f.to(self.device, non_blocking=True) if isinstance(f, torch.Tensor) else f for f in feeds]
            outs = self._finish(self.program.run(dev_feeds))
            return [o.cpu() if isinstance(o, torch.Tensor) else o for o in outs]

    def _bucket(self, n: int) -> Optional[int]:
        for b in self.buckets:
            if b >= n:
                return b
        return None

    def _pick_lane(self) -> _Lane:
        with self._rr_lock:
            lane = self.lanes[self._rr % len(self.lanes)]
            self._rr += 1
        return lane

    def _capture(self, lane: _Lane, b: int) -> None:
        dev = self.device
        ins = []
        hosts = []
        for s in self.in_specs:
            shape = [b] + list(s.shape[1:])
            tdt = T.np_dtype(s.dtype)
            t = torch.zeros(shape, dtype=torch.from_numpy(np.zeros(0, tdt)).dtype, device=dev)
            ins.append(t)
            hosts.append(torch.zeros(shape, dtype=t.dtype, pin_memory=True))
        # eager warm-up on the lane's stream (autotunes kernel tiles for this shape)
        with torch.cuda.stream(lane.stream):
            self._finish(self.program.run(ins))
            self._finish(self.program.run(ins))
        lane.stream.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=lane.stream):
            outs = self._finish(self.program.run(ins))
        lane.graphs[b] = graph
        lane.static_in[b] = ins
        lane.static_out[b] = outs
        lane.host_in[b] = hosts
        lane.host_out[b] = [torch.empty(o.shape, dtype=o.dtype, pin_memory=True) for o in outs]
        log.info("captured HIP graph: %s bucket=%d (%d steps)", self.servable.name, b, len(self.program.steps))

    # ------------------------------------------------------------ run
    def run(self, inputs: Sequence) -> List:
        if not self.use_graphs:
            feeds = [v if (isinstance(v, np.ndarray) and v.dtype == object) or isinstance(v, torch.Tensor)
                     else self._to_device_dtype(s, v) for s, v in zip(self.in_specs, inputs)]
            return self._eager(feeds)
        n = int(inputs[0].shape[0])
        for v in inputs:
            if int(v.shape[0]) != n:
                raise E.invalid("all inputs must have the same batch size (dim 0)")
        b = self._bucket(n)
        if b is None:
            # larger than the biggest bucket: split into bucket-sized chunks
            big = self.buckets[-1]
            parts = [self.run([v[i:i + big] for v in inputs]) for i in range(0, n, big)]
            return [np.concatenate([p[k] for p in parts]) for k in range(len(self.out_specs))]
        lane = self._pick_lane()
        with lane.lock:
            if b not in lane.graphs:
                with torch.cuda.device(self.device):
                    self._capture(lane, b)
            hin, sin = lane.host_in[b], lane.static_in[b]
            for h, v, s in zip(hin, inputs, self.in_specs):
                src = v if isinstance(v, torch.Tensor) else self._to_device_dtype(s, v)
                h[:n].copy_(src.reshape(h[:n].shape))
            with torch.cuda.stream(lane.stream):
                for h, d in zip(hin, sin):
                    d.copy_(h, non_blocking=True)
                lane.graphs[b].replay()
                for so, ho in zip(lane.static_out[b], lane.host_out[b]):
                    ho.copy_(so, non_blocking=True)
            lane.stream.synchronize()
            return [ho[:n].numpy().copy() if ho.dim() else ho.numpy().copy() for ho in lane.host_out[b]]
