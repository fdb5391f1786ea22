"""Persistent dataflow execution of a conv chain (``_FlowBlock``, kernels/flow.hip).

A small-batch ResNet forward is ~50 dependent convolutions, each far too small
to fill 256 CUs: at batch 1 the HIP-graph replay is a latency chain of 58
dispatches of 4.7-11 us (``profiles/round2/r50_b1_replay_stempool.txt``), i.e.
the dependent-kernel boundary plus each kernel's own fill and drain, paid 58
times.  ``fuse_flow`` replaces the maximal run of fused conv ops between the
stem and the classifier head (``_FusedConv2D`` / ``_FusedDualConv`` /
``_ChainConv``) with ONE ``_FlowBlock`` node.  For batches up to
``TFSERVE_FLOW_MAX_BATCH`` it runs as one persistent launch (``hip().flow_run``):
workgroups pull (layer, 32x64 tile, K-slice) tasks in program order, prefetch
the task's weights while the producers finish, wait on per-layer tile counters
and publish their own tiles (see kernels/flow.h).  Larger batches -- and any
CPU run -- execute the member ops one by one, exactly as without the pass.

The launch reads a per-(batch, weights) step table built on the first eager
call (never during a HIP-graph capture, which only replays a cached table):
every activation pointer in it is an offset into a per-call arena, the chain's
input or its output, so a captured graph re-binds them per capture.

SURVEY.md S7/S8 (executor, kernels); the request it serves is the reference
client's batch-1 ResNet Predict (/root/reference/src/lib.rs:229-257).
"""
from __future__ import annotations

import copy
import os
import threading
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from . import ops as O
from .fused import BF16, ChainConv, FusedConv, FusedDualConv, _Ctx, _impl_op, _merge_ctrl

MAX_STEPS = 64                  # kernels/flow.h kFlowMaxSteps
STEP_INTS = 48                  # sizeof(FlowStep) / 4
TILE_M, TILE_N, KT = 32, 64, 64
REF_SHIFT = 60
K_ARENA, K_ENTRY, K_OUT, K_ABS = 0, 1, 2, 3
NULL_REF = K_ABS << REF_SHIFT
CTRL_HEAD = 4                   # ticket, exit count, error flag, epoch
ROW_STRIDE = 16                 # kernels/flow.h kFlowRowStride
MODE_DENSE, MODE_IM2COL, MODE_DUAL = 0, 1, 2
_ALIGN = 256


def max_batch() -> int:
    """Largest batch that runs as one persistent launch (TFSERVE_FLOW_MAX_BATCH;
    larger batches run the block's member ops one by one)."""
    return int(os.environ.get("TFSERVE_FLOW_MAX_BATCH", "4"))


def _ref(kind: int, off: int) -> int:
    return (kind << REF_SHIFT) | int(off)


def _abs(t: Optional[torch.Tensor]) -> int:
    return NULL_REF if t is None else _ref(K_ABS, t.data_ptr())


def conv_flow_ok(impl) -> bool:
    """A fused conv the flow kernel runs: bf16 NHWC with 64-multiple input
    channels (one k-tile = one filter tap x 64 channels), no v2 second output."""
    if isinstance(impl, FusedConv):
        return (impl.use_hip and not impl.c4 and impl.post is None and impl.cin % 64 == 0 and
                impl.cout % 8 == 0 and impl.kh * impl.kw <= 32)
    if isinstance(impl, FusedDualConv):
        return impl.use_hip and impl.post is None and impl.c1 % 64 == 0 and impl.c2 % 64 == 0 and impl.cout % 8 == 0
    if isinstance(impl, ChainConv):
        return conv_flow_ok(impl.a) and conv_flow_ok(impl.b)
    return False


def _n_steps(impl) -> int:
    return 2 if isinstance(impl, ChainConv) else 1


def pick_splits(tiles: int, nk: int, target: int) -> Tuple[int, int]:
    """(splits, k-tiles per split): K-slices until the layer has ~``target``
    tasks, keeping at least two k-tiles per slice."""
    s = 1
    cap = int(os.environ.get("TFSERVE_FLOW_MAX_SPLITS", "1"))
    while s < cap and tiles * s * 2 <= target and nk // (s * 2) >= 2:
        s *= 2
    per = -(-nk // s)
    return -(-nk // per), per


class FlowBlock:
    """A chain of fused convs (``subs``: (impl, node, input value ids, output
    value ids) in program order; value 0 is the chain's input) with one
    output value ``exit_id``."""

    def __init__(self, subs, exit_id: int, name: str):
        self.subs = subs
        self.exit_id = exit_id
        self.name = name
        self.children = tuple(f"sub{i}" for i in range(len(subs)))
        for i, (impl, _n, _i, _o) in enumerate(subs):
            setattr(self, f"sub{i}", impl)
        self.use_hip = all(getattr(impl, "use_hip", False) for impl, _n, _i, _o in subs)
        # last reader of each value (the sequential path frees it after that sub)
        last: Dict[int, int] = {}
        for i, (_impl, _n, ins, _outs) in enumerate(subs):
            for v in ins:
                last[v] = i
        self._free_after: List[List[int]] = [[] for _ in subs]
        for v, i in last.items():
            if v not in (0, exit_id):
                self._free_after[i].append(v)
        self._tables: Dict[tuple, dict] = {}
        self._lock = threading.Lock()
        self._warned = False

    # ---- sequential path (large batches, CPU)
    def run_sequential(self, ctx, x):
        vals = {0: x}
        for (impl, node, ins, outs), dead in zip(self.subs, self._free_after):
            res = impl(ctx, node, [vals[v] for v in ins])
            for v, o in zip(outs, res):
                vals[v] = o
            for v in dead:
                vals.pop(v, None)
        return vals[self.exit_id]

    # ---- step list (host side; no device work)
    def steps(self, x_shape) -> List[dict]:
        """Expand the subs into kernel steps with their NHWC geometry."""
        shapes = {0: tuple(int(s) for s in x_shape)}
        out = []
        for impl, _node, ins, outs in self.subs:
            if isinstance(impl, ChainConv):
                out.append(self._conv_step(impl.a, ins[0], ins[1] if len(ins) > 1 else None, outs[0], shapes))
                out.append(self._conv_step(impl.b, outs[0], None, outs[1], shapes))
            elif isinstance(impl, FusedDualConv):
                h, x = shapes[ins[0]], shapes[ins[1]]
                n, ho, wo, c1 = h
                if c1 != impl.c1 or x[3] != impl.c2 or (x[1] - 1) // impl.sh + 1 != ho or \
                        (x[2] - 1) // impl.sw + 1 != wo:
                    raise O.Unsupported("flow: dual conv operand shapes")
                shapes[outs[0]] = (n, ho, wo, impl.cout)
                out.append(dict(impl=impl, mode=MODE_DUAL, a=ins[0], a2=ins[1], res=None, out=outs[0],
                                M=n * ho * wo, N=impl.cout, K=impl.c1 + impl.c2, K1=impl.c1, lda=impl.c1,
                                ldb=int(impl.w.shape[1]), H=x[1], W=x[2], C=impl.c2, Ho=ho, Wo=wo, KH=1, KW=1,
                                SH=impl.sh, SW=impl.sw, PT=0, PL=0, w=impl.w, bias=impl.b, act=O_ACT(impl.act)))
            else:
                out.append(self._conv_step(impl, ins[0], ins[1] if len(ins) > 1 else None, outs[0], shapes))
        return out

    @staticmethod
    def _conv_step(impl: FusedConv, a: int, res: Optional[int], o: int, shapes) -> dict:
        n, h, w, c = shapes[a]
        if c != impl.cin:
            raise O.Unsupported("flow: conv input channels")
        pt, pb, pl, pr = impl.pads_for(h, w)
        ho = (h + pt + pb - impl.kh) // impl.sh + 1
        wo = (w + pl + pr - impl.kw) // impl.sw + 1
        shapes[o] = (n, ho, wo, impl.cout)
        if res is not None and shapes[res] != shapes[o]:
            raise O.Unsupported("flow: residual shape")
        dense = impl.kh == impl.kw == impl.sh == impl.sw == 1 and not (pt or pb or pl or pr)
        return dict(impl=impl, mode=MODE_DENSE if dense else MODE_IM2COL, a=a, a2=None, res=res, out=o,
                    M=n * ho * wo, N=impl.cout, K=impl.kh * impl.kw * c, K1=0, lda=c, ldb=int(impl.w.shape[1]),
                    H=h, W=w, C=c, Ho=ho, Wo=wo, KH=impl.kh, KW=impl.kw, SH=impl.sh, SW=impl.sw, PT=pt, PL=pl,
                    w=impl.w, bias=impl.b, act=O_ACT(impl.act))

    def build_table(self, x_shape, target_tasks: int) -> dict:
        """The kernel's step table (int32 numpy) + arena / ctrl sizes."""
        steps = self.steps(x_shape)
        if len(steps) > MAX_STEPS:
            raise O.Unsupported(f"flow: {len(steps)} steps > {MAX_STEPS}")
        producer = {s["out"]: i for i, s in enumerate(steps)}
        nbytes = {0: int(np.prod(x_shape)) * 2}
        arena, off = 0, {}
        exit_shape = None
        for s in steps:
            size = s["M"] * s["N"] * 2
            nbytes[s["out"]] = size
            if s["out"] == self.exit_id:
                exit_shape = (s["M"], s["N"])
            else:
                off[s["out"]] = arena
                arena += -(-size // _ALIGN) * _ALIGN
        if exit_shape is None:
            raise O.Unsupported("flow: the exit value is not produced by a step")

        def vref(v):
            if v is None:
                return NULL_REF
            if v == 0:
                return _ref(K_ENTRY, 0)
            if v == self.exit_id:
                return _ref(K_OUT, 0)
            return _ref(K_ARENA, off[v])

        tab = np.zeros(MAX_STEPS + len(steps) * STEP_INTS, dtype=np.int32)
        tab[:MAX_STEPS] = np.iinfo(np.int32).max
        layout = []
        for s in steps:
            ntm, ntn = -(-s["M"] // TILE_M), -(-s["N"] // TILE_N)
            splits, per = pick_splits(ntm * ntn, s["K"] // KT, target_tasks)
            layout.append((ntm, ntn, splits, per))
        # control words: the head, the split-K arrival counters, the row-block counters
        ctr = CTRL_HEAD
        ctrs = []
        for ntm, ntn, splits, _per in layout:
            ctrs.append(ctr if splits > 1 else 0)
            ctr += ntm * ntn if splits > 1 else 0
        ctr = -(-ctr // ROW_STRIDE) * ROW_STRIDE
        task0 = 0
        for i, (s, (ntm, ntn, splits, per)) in enumerate(zip(steps, layout)):
            ws = NULL_REF
            if splits > 1:
                ws = _ref(K_ARENA, arena)
                arena += -(-(splits * s["M"] * s["N"] * 4) // _ALIGN) * _ALIGN
            ntasks = ntm * ntn * splits
            deps = [producer.get(v, -1) if v is not None else -1 for v in (s["a"], s["a2"], s["res"])]
            rctr = ctr
            ctr += ntm * ROW_STRIDE
            refs = [vref(s["a"]), vref(s["a2"]), _abs(s["w"]), _abs(s["bias"]), vref(s["res"]), vref(s["out"]),
                    ws, 0]
            ints = [s["M"], s["N"], s["K"], s["K1"], s["lda"], s["ldb"], s["H"], s["W"], s["C"], s["Ho"], s["Wo"],
                    s["KH"], s["KW"], s["SH"], s["SW"], s["PT"], s["PL"], s["mode"], s["act"], ntm, ntn, splits, per,
                    ntasks, deps[0], deps[1], deps[2], ctrs[i], nbytes[s["a"]],
                    nbytes[s["a2"]] if s["a2"] is not None else 0, int(s["w"].numel()) * 2, rctr]
            base = MAX_STEPS + i * STEP_INTS
            tab[base:base + 16] = np.array(refs, dtype=np.int64).view(np.int32)
            tab[base + 16:base + STEP_INTS] = np.array(ints, dtype=np.int64).astype(np.int32)
            tab[i] = task0
            s.update(ntm=ntm, ntn=ntn, splits=splits, ktps=per, ntasks=ntasks, task0=task0, deps=deps, rctr=rctr)
            task0 += ntasks
        n_out = exit_shape[0] * exit_shape[1]
        return dict(table=tab, nsteps=len(steps), ntasks=task0, arena=max(arena, _ALIGN), ctrl_ints=ctr,
                    steps=steps, out_elems=n_out)

    # ---- persistent path
    def _key(self, x) -> tuple:
        ptrs = []
        for st_impl, _n, _i, _o in self.subs:
            for impl in ((st_impl.a, st_impl.b) if isinstance(st_impl, ChainConv) else (st_impl,)):
                ptrs += [impl.w.data_ptr(), impl.b.data_ptr()]
        return (tuple(x.shape), x.device.index, tuple(ptrs))

    def table_for(self, x) -> Optional[dict]:
        key = self._key(x)
        hit = self._tables.get(key)
        if hit is not None or torch.cuda.is_current_stream_capturing():
            return hit
        with self._lock:
            hit = self._tables.get(key)
            if hit is None:
                props = torch.cuda.get_device_properties(x.device)
                cus = int(getattr(props, "multi_processor_count", 256))
                target = int(os.environ.get("TFSERVE_FLOW_TARGET", str(cus)))
                hit = self.build_table(tuple(x.shape), target_tasks=target)
                hit["table_dev"] = torch.from_numpy(hit["table"]).to(x.device)
                mult = float(os.environ.get("TFSERVE_FLOW_GRID_MULT", "1"))
                hit["grid"] = max(1, min(hit["ntasks"], int(cus * mult)))
                last = next(s for s in hit["steps"] if s["out"] == self.exit_id)
                hit["out_shape"] = (int(x.shape[0]), last["Ho"], last["Wo"], last["N"])
                self._tables[key] = hit
        return hit

    def enabled_for(self, x) -> bool:
        return (self.use_hip and isinstance(x, torch.Tensor) and x.is_cuda and x.dim() == 4 and
                x.dtype == BF16 and x.shape[0] <= max_batch())

    def run_flow(self, x, ctrl: Optional[torch.Tensor] = None):
        """One persistent launch.  ``ctrl``: zeroed int32 control words (the
        row-block counters count across launches, so a caller that passes its
        own keeps it for its launches only); None: a fresh zeroed block
        eagerly, a permanent pool slice inside a HIP-graph capture."""
        from ..ops import hip
        tab = self.table_for(x)
        if tab is None:
            return None
        x = x.contiguous()
        if ctrl is None and not torch.cuda.is_current_stream_capturing():
            ctrl = torch.zeros(tab["ctrl_ints"], dtype=torch.int32, device=x.device)
        out = torch.empty(tab["out_shape"], device=x.device, dtype=BF16)
        arena = torch.empty(tab["arena"], device=x.device, dtype=torch.uint8)
        hip().flow_run(tab["table_dev"], tab["nsteps"], tab["ntasks"], arena, x, out, tab["ctrl_ints"],
                       tab["grid"], ctrl)
        return out

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if self.enabled_for(x):
            y = self.run_flow(x)
            if y is not None:
                return [y]
            if not self._warned:
                self._warned = True
                import logging
                logging.getLogger("tfserve.gpu").warning(
                    "flow block %s: no step table for batch %d at capture time; running its ops one by one",
                    self.name, int(x.shape[0]))
        return [self.run_sequential(ctx, x)]


def O_ACT(act: str) -> int:
    from ..ops import ACT
    return int(ACT[act])


O.OPS["_FlowBlock"] = _impl_op

_FLOW_OPS = ("_FusedConv2D", "_FusedDualConv", "_ChainConv")


def _region(g, c: _Ctx, names: List[str]):
    """(entry ref, exit ref) when ``names`` reads exactly one outside value and
    exactly one of its values is used outside (or fetched), else None."""
    inside = set(names)
    entries = set()
    for nm in names:
        for r in g.nodes[nm].inputs:
            if r[0] not in inside:
                entries.add(tuple(r))
    exits = set()
    for nm in names:
        for cn, _pos, oi in c.cons.get(nm, []):
            if cn not in inside:
                exits.add((nm, oi))
    if len(entries) != 1 or len(exits) != 1:
        return None
    return next(iter(entries)), next(iter(exits))


def fuse_flow(g, order, fed, fetch_refs, device, opts):
    """Maximal runs of flow-capable fused convs (consecutive in program order,
    one input, one output) -> ``_FlowBlock``.  Opt-in (TFSERVE_FLOW=1 on GPU
    programs; ``force`` builds it on CPU too, where it runs sequentially): on
    MI355X the one-launch chain measured slower than the HIP-graph launch
    chain it replaces at every batch (b1 0.417 vs 0.387 ms at its best knobs,
    profiles/round3/flow.md), so the default program keeps the per-layer
    kernels."""
    mode = os.environ.get("TFSERVE_FLOW", "0")
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    if mode == "0" or (not c.use_hip and mode != "force"):
        return
    runs, cur = [], []
    for name in order:
        n = g.nodes.get(name)
        ok = (n is not None and n.op in _FLOW_OPS and name not in c.fetch_nodes and
              (conv_flow_ok(n.attrs.get("_impl")) or (mode == "force" and not c.use_hip)))
        if ok:
            cur.append(name)
        else:
            if len(cur) >= 2:
                runs.append(cur)
            cur = []
    if len(cur) >= 2:
        runs.append(cur)
    for run in runs:
        while len(run) >= 2:
            # longest prefix within the step budget that is a one-in / one-out region
            total, end = 0, 0
            for i, nm in enumerate(run):
                total += _n_steps(g.nodes[nm].attrs["_impl"])
                if total > MAX_STEPS:
                    break
                end = i + 1
            chunk, reg = run[:end], None
            while len(chunk) >= 2:
                reg = _region(g, c, chunk)
                if reg is not None:
                    break
                chunk = chunk[:-1]
            if reg is None or len(chunk) < 2:
                run = run[1:]
                continue
            _make_block(g, chunk, reg)
            c.refresh()
            run = run[len(chunk):]


def _make_block(g, names: List[str], reg) -> None:
    entry, exit_ref = reg
    ids = {tuple(entry): 0}
    subs = []
    for nm in names:
        n = g.nodes[nm]
        impl = n.attrs["_impl"]
        ins = [ids[tuple(r)] for r in n.inputs]
        n_out = 2 if isinstance(impl, ChainConv) else 1
        outs = []
        for oi in range(n_out):
            ids[(nm, oi)] = len(ids)
            outs.append(ids[(nm, oi)])
        subs.append((impl, copy.copy(n), ins, outs))   # (the kept node becomes the block)
    block = FlowBlock(subs, ids[tuple(exit_ref)], names[0] + "/flow")
    nodes = [g.nodes[nm] for nm in names]
    keep = g.nodes[exit_ref[0]]
    ctrl = _merge_ctrl(nodes)
    # consumers of the exit value now read output 0 of the kept node
    for n in g.nodes.values():
        if n.name in names:
            continue
        n.inputs = [(keep.name, 0) if tuple(r) == tuple(exit_ref) else r for r in n.inputs]
    for nm in names:
        if nm != keep.name:
            del g.nodes[nm]
    keep.op = "_FlowBlock"
    keep.inputs = [tuple(entry)]
    keep.ctrl = ctrl
    keep.attrs = {"_impl": block}
    keep.value = None
