"""A loaded model version ("servable") and its signature runners.

A :class:`Servable` owns one SavedModel version on one device.  Each distinct
(signature, fed aliases, fetched aliases) combination is compiled once into a
:class:`~..graph.compiler.Program` by a :class:`Runner`; the GPU runtime
(``server/gpu_runtime.py``) adds fused HIP kernels, bf16 weights and HIP-graph
capture per batch bucket on top of the same interface.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..graph import ops as O
from ..graph.compiler import CompileError, Program, bind_variables, compile_program
from ..graph.ir import from_graph_def
from ..savedmodel import saved_model as sm
from ..utils import tensors as T
from . import errors as E

DEFAULT_SIGNATURE = "serving_default"
PREDICT_METHOD = "tensorflow/serving/predict"
CLASSIFY_METHOD = "tensorflow/serving/classify"
REGRESS_METHOD = "tensorflow/serving/regress"


@dataclass
class ServableOptions:
    device: str = "cpu"
    fuse: Optional[bool] = None          # default: on for GPU devices
    compute_dtype: str = "bf16"          # bf16 on GPU (fp32 on CPU always)
    hip_graphs: bool = True
    graph_autotune: bool = True          # re-pick GEMM tiles by timing whole-graph replays (ops.graph_tune)
    lanes: int = 4                       # GPU lanes = fast-path batch slots (stream + pinned staging + graphs)
    max_batch_size: int = 32
    allowed_batch_sizes: Tuple[int, ...] = ()
    warmup: bool = True
    verify_checksums: bool = True
    extra: dict = field(default_factory=dict)

    @property
    def torch_device(self) -> torch.device:
        return torch.device(self.device)

    @property
    def is_gpu(self) -> bool:
        return self.torch_device.type == "cuda"


@dataclass
class TensorSpec:
    alias: str
    name: str
    dtype: int
    shape: Optional[List[int]]   # None = unknown rank


def _specs(m) -> Dict[str, TensorSpec]:
    out = {}
    for alias, ti in m.items():
        shape = None if ti.tensor_shape.unknown_rank else [d.size for d in ti.tensor_shape.dim]
        if ti.WhichOneof("encoding") != "name":
            raise E.unimplemented(f"sparse TensorInfo for {alias!r} is not supported")
        out[alias] = TensorSpec(alias, ti.name, ti.dtype, shape)
    return out


class Runner:
    """Executes a fixed feed/fetch set of one signature (eager interpreter)."""

    def __init__(self, servable: "Servable", in_specs: List[TensorSpec], out_specs: List[TensorSpec]):
        self.servable = servable
        self.in_specs = in_specs
        self.out_specs = out_specs
        g = servable.fresh_graph()
        passes = servable.passes()
        self.program: Program = compile_program(
            g, [s.name for s in in_specs], [s.name for s in out_specs],
            servable.options.torch_device, passes, servable.options.extra)
        share_weights(servable, in_specs, out_specs, self.program)

    def run(self, inputs: Sequence) -> List:
        dev = self.servable.options.torch_device
        feeds = []
        for spec, v in zip(self.in_specs, inputs):
            if isinstance(v, np.ndarray) and v.dtype == object:
                feeds.append(v)
                continue
            t = v if isinstance(v, torch.Tensor) else _np_to_torch(v, spec.dtype)
            if dev.type != "cpu":
                t = t.to(dev, non_blocking=True)
            feeds.append(t)
        return self.program.run(feeds)


def runner_key(in_specs, out_specs) -> str:
    return "|".join(s.name for s in in_specs) + ">" + "|".join(s.name for s in out_specs)


def share_weights(servable, in_specs, out_specs, program) -> None:
    """Replicas: the leader broadcasts ``program``'s packed device weights; a
    follower (compiled on shapes only) binds them (parallel/weights.py)."""
    src = getattr(servable, "weight_source", None)
    if src is None:
        return

    def recompile():
        real = sm.load(servable.path, verify=servable.options.verify_checksums)
        g = from_graph_def(real.graph_def)
        bind_variables(g, real.bundle)
        servable.bundle = real
        return compile_program(g, [s.name for s in in_specs], [s.name for s in out_specs],
                               servable.options.torch_device, servable.passes(), servable.options.extra)
    src.share_program(servable.name, servable.version, runner_key(in_specs, out_specs), program, recompile)


def _np_to_torch(a: np.ndarray, dt: int) -> torch.Tensor:
    if dt == T.DT_BFLOAT16:
        return torch.from_numpy(np.require(a, requirements="C").view(np.int16)).view(torch.bfloat16)
    if not a.flags.writeable:
        # zero-copy views into request bytes are read-only; torch wants writable
        return torch.from_numpy(np.array(a))
    return torch.from_numpy(np.require(a, requirements="C"))


def to_numpy(v) -> np.ndarray:
    if isinstance(v, np.ndarray):
        return v
    if isinstance(v, torch.Tensor):
        v = v.detach()
        if v.dtype == torch.bfloat16:
            return v.cpu().view(torch.int16).numpy().view(np.uint16)
        return v.cpu().numpy()
    return np.asarray(v)


class Servable:
    """One loaded version of one model."""

    def __init__(self, name: str, version: int, path: str, options: ServableOptions,
                 bundle: Optional[sm.SavedModelBundle] = None, weight_source=None):
        self.name = name
        self.version = version
        self.path = path
        self.options = options
        # parallel/weights.py ReplicatedWeightSource: compiled programs share
        # the leader's device weight blob (a follower's bundle is shape-only)
        self.weight_source = weight_source
        self.bundle = bundle or sm.load(path, verify=options.verify_checksums)
        self.signatures = self.bundle.signatures
        self._runners: Dict[tuple, Runner] = {}
        self._by_tensors: Dict[str, Runner] = {}
        self._lock = threading.Lock()
        self.in_flight = 0
        self._cv = threading.Condition()
        self.loaded_at = time.time()
        from ..utils.faults import FaultPoint
        fp = FaultPoint()
        self.fault = fp if fp.enabled else None     # TFSERVE_FAULT injection (tests)
        self._graph_lock = threading.Lock()

    # ------------------------------------------------------------ graph helpers
    def fresh_graph(self):
        with self._graph_lock:
            g = from_graph_def(self.bundle.graph_def)
            bind_variables(g, self.bundle.bundle)
        return g

    def passes(self):
        use = self.options.fuse if self.options.fuse is not None else self.options.is_gpu
        if not use:
            return ()
        from ..graph import fused
        return fused.default_passes(self.options)

    # ------------------------------------------------------------ signatures
    def signature(self, name: str):
        key = name or DEFAULT_SIGNATURE
        sig = self.signatures.get(key)
        if sig is None:
            raise E.invalid(f'Serving signature key "{key}" not found.')
        return key, sig

    def runner(self, sig_name: str, in_aliases: Sequence[str], out_aliases: Sequence[str]) -> Runner:
        key = (sig_name, tuple(in_aliases), tuple(out_aliases))
        r = self._runners.get(key)
        if r is not None:
            return r
        with self._lock:
            r = self._runners.get(key)
            if r is None:
                _k, sig = self.signature(sig_name)
                ins, outs = _specs(sig.inputs), _specs(sig.outputs)
                in_specs, out_specs = [ins[a] for a in in_aliases], [outs[a] for a in out_aliases]
                # alias sets that name the same tensors (warm-up's sorted outputs,
                # a request's filter) share ONE runner: one compile, one set of
                # captured graphs, one weight broadcast between replicas
                tkey = runner_key(in_specs, out_specs)
                r = self._by_tensors.get(tkey)
                if r is None:
                    try:
                        r = self._make_runner(in_specs, out_specs)
                    except CompileError as e:
                        raise E.ServingError(E.INVALID_ARGUMENT if "not found" in str(e) else E.UNIMPLEMENTED,
                                             str(e)) from None
                    self._by_tensors[tkey] = r
                self._runners[key] = r
        return r

    def _make_runner(self, in_specs, out_specs) -> Runner:
        if self.options.is_gpu:
            from .gpu_runtime import GpuRunner
            return GpuRunner(self, in_specs, out_specs, lanes=self.options.lanes)
        r = Runner(self, in_specs, out_specs)
        from . import cpu_runtime
        if self.options.lanes > 0 and cpu_runtime.batched(in_specs, out_specs):
            return cpu_runtime.CpuRunner(r, lanes=min(self.options.lanes, 2))   # batched native fast path
        return r

    def input_specs(self, sig_name: str) -> Dict[str, TensorSpec]:
        return _specs(self.signature(sig_name)[1].inputs)

    def output_specs(self, sig_name: str) -> Dict[str, TensorSpec]:
        return _specs(self.signature(sig_name)[1].outputs)

    # ------------------------------------------------------------ execution
    def run(self, sig_name: str, inputs: Dict[str, object], out_aliases: Sequence[str]) -> Dict[str, np.ndarray]:
        in_aliases = sorted(inputs)
        r = self.runner(sig_name, in_aliases, list(out_aliases))
        self.acquire()
        try:
            try:
                outs = r.run([inputs[a] for a in in_aliases])
            except O.OpError as e:
                raise E.invalid(str(e)) from None
            except O.Unsupported as e:
                raise E.unimplemented(str(e)) from None
        finally:
            self.release()
        return {a: to_numpy(v) for a, v in zip(out_aliases, outs)}

    # ------------------------------------------------------------ refcount for safe unload
    def acquire(self):
        with self._cv:
            self.in_flight += 1

    def release(self):
        with self._cv:
            self.in_flight -= 1
            if self.in_flight == 0:
                self._cv.notify_all()

    def drain(self, timeout: float = 30.0) -> bool:
        deadline = time.time() + timeout
        with self._cv:
            while self.in_flight > 0:
                left = deadline - time.time()
                if left <= 0:
                    return False
                self._cv.wait(left)
        return True

    def warmup(self):
        """Compile + run the default predict signature once on zeros (static shapes only)."""
        if not self.options.warmup:
            return
        for key, sig in self.signatures.items():
            if sig.method_name != PREDICT_METHOD:
                continue
            ins = _specs(sig.inputs)
            feeds = {}
            ok = True
            for a, s in ins.items():
                if s.shape is None or s.dtype == T.DT_STRING:
                    ok = False
                    break
                shape = [1 if d < 0 else d for d in s.shape]
                feeds[a] = np.zeros(shape, dtype=T.np_dtype(s.dtype))
            if ok:
                try:
                    self.run(key, feeds, sorted(_specs(sig.outputs)))
                except E.ServingError:
                    pass
            break

    def unload(self):
        self._runners.clear()
        self._by_tensors.clear()
        self.bundle = None
        if self.options.is_gpu:
            from .gpu_runtime import CAPTURE_LOCK
            with CAPTURE_LOCK:   # never while another servable captures its graphs
                torch.cuda.empty_cache()
