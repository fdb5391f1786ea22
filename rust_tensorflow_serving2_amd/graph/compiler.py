"""GraphDef -> executable Program.

Pipeline (per signature, per feed/fetch set):

1. **bind variables** — ``VariableV2`` / ``VarHandleOp`` nodes become constants
   loaded from the TensorBundle (key = node name / ``shared_name``);
2. **prune** to the sub-graph that the fetches need, with fed tensors as leaves
   (feeding an interior tensor overrides its producer, as in TF);
3. **constant-fold** everything that does not depend on a feed;
4. **fusion passes** (``graph/fused.py``): Conv+BN(+residual)(+ReLU) folding,
   MatMul+BiasAdd(+act), LayerNorm/GELU/attention pattern matching, softmax+argmax
   — rewritten into fused ops that run as hand-written HIP kernels on MI355X;
5. **placement** — weights to the device (bf16 for fused MFMA ops), shape
   arithmetic stays on the host so a Program can be captured in a HIP graph;
6. **linearise** into a list of steps over value slots.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch

from ..utils import tensors as T
from . import ops as O
from .placement import to_device
from .ir import Graph, Node, fmt_ref, parse_ref

NON_FOLDABLE = {"Placeholder", "PlaceholderWithDefault", "ParseExample", "ParseExampleV2", "NoOp",
                "RandomUniform", "RandomStandardNormal", "TruncatedNormal", "VariableV2",
                "VarHandleOp", "SaveV2", "RestoreV2", "Assign", "AssignVariableOp"}
MAX_FOLD_ELEMS = 1 << 26


class CompileError(ValueError):
    pass


def const_value(node: Node):
    """Decode a Const node's value into a torch tensor (or numpy object array)."""
    v = node.attrs.get("value")
    dt = node.attrs.get("dtype", T.DT_FLOAT)
    if isinstance(v, np.ndarray) and v.dtype == object:
        return v
    a = np.asarray(v)
    if dt == T.DT_BFLOAT16:
        return torch.from_numpy(a.astype(np.uint16).view(np.int16).copy()).view(torch.bfloat16)
    if dt == T.DT_STRING:
        return a.astype(object)
    t = torch.from_numpy(np.array(a, copy=True))
    want = O.DT_TO_TORCH.get(dt)
    if want is not None and t.dtype != want:
        t = t.to(want)
    return t


def array_to_value(a: np.ndarray, dt: int):
    if isinstance(a, torch.Tensor):      # a meta (shape-only) weight: parallel/weights.py followers
        return a
    if dt == T.DT_BFLOAT16:
        return torch.from_numpy(np.array(a, dtype=np.uint16).view(np.int16)).view(torch.bfloat16)
    if dt == T.DT_STRING:
        return np.asarray(a, dtype=object)
    return torch.from_numpy(np.array(a, copy=True))


def bind_variables(g: Graph, bundle) -> None:
    from .ir import restore_keys
    keys = restore_keys(g) if bundle is not None else {}
    for node in list(g.nodes.values()):
        if node.op in ("VariableV2", "Variable", "VarHandleOp"):
            key = node.name
            if node.name in keys and keys[node.name] in bundle:
                key = keys[node.name]          # saver graph (TF2 object-path keys)
            elif node.op == "VarHandleOp":
                sn = node.sattr("shared_name")
                if sn and bundle is not None and sn in bundle:
                    key = sn
            if bundle is None or key not in bundle:
                continue  # left unbound: error only if it is actually needed
            dt = bundle.dtype(key)
            node.value = [array_to_value(bundle[key], dt)]
            node.op = "Const"
            node.attrs = {"dtype": dt, "_variable": key}


class Program:
    """A linearised, device-placed computation (feeds -> fetches)."""

    def __init__(self, steps, n_slots, feed_slots, fetch_slots, const_slots, device, feed_dtypes,
                 graph: Graph, order: List[str]):
        self.steps = steps
        self.n_slots = n_slots
        self.feed_slots = feed_slots
        self.fetch_slots = fetch_slots
        self.const_slots = const_slots
        self.device = device
        self.feed_dtypes = feed_dtypes
        self.graph = graph
        self.order = order
        self._ctx = O.Ctx(device)
        self.free_after = plan_release(steps, n_slots, feed_slots, fetch_slots, const_slots)

    def run(self, feeds: Sequence) -> List:
        vals: List = [None] * self.n_slots
        for slot, v in self.const_slots:
            vals[slot] = v
        for slot, v in zip(self.feed_slots, feeds):
            vals[slot] = v
        ctx = self._ctx
        for (fn, node, in_slots, out_slots), dead in zip(self.steps, self.free_after):
            try:
                outs = fn(ctx, node, [vals[s] for s in in_slots])
            except (O.OpError, O.Unsupported):
                raise
            except (RuntimeError, ValueError, IndexError, TypeError) as e:
                raise O.OpError(f"{node.op} node '{node.name}': {e}") from e
            for s, o in zip(out_slots, outs):
                if s >= 0:
                    vals[s] = o
            # activation memory plan: drop every value whose last reader was
            # this step, so the allocator (and a HIP-graph capture's pool)
            # reuses its block for later steps -- peak-live instead of the sum
            # of all activations per captured graph
            for s in dead:
                vals[s] = None
        return [vals[s] for s in self.fetch_slots]

    def activation_plan(self) -> Dict[str, int]:
        """Values alive at once: peak under the release plan vs all computed."""
        produced = sum(1 for _f, _n, _i, outs in self.steps for s in outs if s >= 0)
        live, peak = 0, 0
        for (_f, _n, _i, outs), dead in zip(self.steps, self.free_after):
            live += sum(1 for s in outs if s >= 0)
            peak = max(peak, live)
            live -= len(dead)
        return {"values": produced, "peak_live_values": peak}

    def feed_accepts_bf16(self, i: int) -> bool:
        """Whether feed ``i`` may be given as bf16 instead of fp32: every step
        that reads it is a fused op that rounds that operand to bf16 itself
        (``accepts_bf16_input``), and the feed is not fetched."""
        slot = self.feed_slots[i]
        if slot in self.fetch_slots:
            return False
        users = [(node, list(ins).index(slot)) for _fn, node, ins, _o in self.steps if slot in ins]
        for node, pos in users:
            impl = node.attrs.get("_impl")
            if impl is None or not getattr(impl, "accepts_bf16_input", lambda _p: False)(pos):
                return False
        return bool(users)

    def op_histogram(self, flat: bool = False) -> Dict[str, int]:
        """Steps per op; ``flat``: count the member ops of block ops (``_FlowBlock``)
        instead of the blocks."""
        h: Dict[str, int] = {}
        for _fn, node, _i, _o in self.steps:
            subs = getattr(node.attrs.get("_impl"), "subs", None) if flat else None
            for op in ([sub[1].op for sub in subs] if subs else [node.op]):
                h[op] = h.get(op, 0) + 1
        return h


def plan_release(steps, n_slots: int, feed_slots, fetch_slots, const_slots) -> List[List[int]]:
    """Per step, the value slots whose last use it is (liveness over the linear
    step list): computed values that are not fetched, plus outputs nobody reads
    (dropped right after their producer).  Feeds and constants belong to the
    caller / the program and are never released."""
    keep = set(fetch_slots) | set(feed_slots) | {s for s, _v in const_slots}
    last: Dict[int, int] = {}
    for i, (_fn, _node, ins, outs) in enumerate(steps):
        for s in outs:
            if s >= 0:
                last.setdefault(s, i)
        for s in ins:
            last[s] = i
    free: List[List[int]] = [[] for _ in steps]
    for s, i in last.items():
        if s not in keep:
            free[i].append(s)
    return free


def _fold(g: Graph, order: List[str], fed: Set[str]) -> None:
    ctx = O.Ctx(torch.device("cpu"))
    for name in order:
        node = g.nodes[name]
        if node.op == "Const":
            if node.value is None:
                node.value = [const_value(node)]
            continue
        if name in fed or node.op in NON_FOLDABLE or node.op not in O.OPS:
            continue
        if node.ctrl and any(g.nodes[c].op != "Const" for c in node.ctrl):
            continue
        if not node.inputs:
            continue
        srcs = [g.nodes[s] for s, _ in node.inputs]
        if not all(s.op == "Const" and s.value is not None and i < len(s.value)
                   for s, (_, i) in zip(srcs, node.inputs)):
            continue
        ins = [s.value[i] for s, (_, i) in zip(srcs, node.inputs)]
        try:
            outs = O.OPS[node.op](ctx, node, ins)
        except Exception:
            continue  # leave it for run time (and run-time error reporting)
        if any(isinstance(o, torch.Tensor) and o.numel() > MAX_FOLD_ELEMS for o in outs):
            continue
        node.value = list(outs)
        node.op = "Const"
        node.inputs = []
        node.ctrl = []


# Pure ops that are safe to merge when they have identical inputs and attrs.
_CSE_OPS = {"Add", "AddV2", "Sub", "Mul", "RealDiv", "Maximum", "Minimum", "Neg", "ExpandDims", "Reshape",
            "Squeeze", "Cast", "Transpose", "StridedSlice", "Identity", "Exp", "Rsqrt", "Sqrt", "Tanh", "Relu",
            "Pow", "SquaredDifference", "Mean", "Sum", "ConcatV2", "Pack", "Shape", "Fill", "Tile", "GatherV2",
            "OneHot", "BiasAdd", "Softmax", "Erf"}


def _attrs_key(attrs) -> Optional[str]:
    try:
        return repr(sorted((k, v) for k, v in attrs.items() if not isinstance(v, torch.Tensor)))
    except TypeError:
        return None


def cse(graph: Graph, order: Sequence[str], fed_nodes: Set[str], fetch_refs) -> int:
    """Common-subexpression elimination: small constants with equal values and
    pure ops with identical (op, inputs, attrs) collapse onto one node.  BERT's
    TF graph, for one, recomputes the attention-mask adder ``(1 - mask) *
    -10000`` in every layer: 12 copies of three elementwise kernels per batch
    become one.  Returns the number of nodes merged."""
    fetch_nodes = {n for n, _ in fetch_refs}
    rep: Dict[str, str] = {}
    seen: Dict[tuple, str] = {}
    for name in order:
        n = graph.nodes[name]
        if rep:
            n.inputs = [(rep.get(s, s), i) for s, i in n.inputs]
            n.ctrl = [rep.get(c, c) for c in n.ctrl]
        if name in fetch_nodes or name in fed_nodes or n.ctrl:
            continue
        key = None
        if n.op == "Const" and not n.attrs.get("_variable"):
            # (model variables are never merged: a replica compiling on shape-only
            # weights must build the same program as the one holding the values)
            v = n.value[0] if n.value else const_value(n)
            if isinstance(v, torch.Tensor) and not v.is_meta and v.numel() <= 64 and \
                    (not n.value or len(n.value) == 1):
                key = ("Const", str(v.dtype), tuple(v.shape), v.detach().cpu().numpy().tobytes())
        elif n.op in _CSE_OPS:
            ak = _attrs_key(n.attrs)
            if ak is not None:
                key = (n.op, tuple(n.inputs), ak)
        if key is None:
            continue
        if key in seen:
            rep[name] = seen[key]
        else:
            seen[key] = name
    if rep:
        # drop the merged duplicates so later passes see the true consumer sets
        for n in graph.nodes.values():
            n.inputs = [(rep.get(s, s), i) for s, i in n.inputs]
            n.ctrl = [rep.get(c, c) for c in n.ctrl]
        for name in rep:
            del graph.nodes[name]
    return len(rep)


def compile_program(graph: Graph, feeds: Sequence[str], fetches: Sequence[str],
                    device: torch.device = torch.device("cpu"), passes: Sequence = (),
                    pass_options: Optional[dict] = None) -> Program:
    feed_refs = [parse_ref(f) for f in feeds]
    fetch_refs = [parse_ref(f) for f in fetches]
    for n, _ in feed_refs + fetch_refs:
        if n not in graph.nodes:
            raise CompileError(f"tensor {n!r} not found in graph")
    fed_nodes = {n for n, _ in feed_refs}
    # a fed node's other outputs are not computable unless all outputs are fed
    order = graph.topo([n for n, _ in fetch_refs], stop=fed_nodes)
    _fold(graph, order, fed_nodes)
    order = graph.topo([n for n, _ in fetch_refs], stop=fed_nodes)
    if cse(graph, order, fed_nodes, fetch_refs):
        order = graph.topo([n for n, _ in fetch_refs], stop=fed_nodes)
    for p in passes:
        p(graph, order, fed_nodes, fetch_refs, device, pass_options or {})
        order = graph.topo([n for n, _ in fetch_refs], stop=fed_nodes)

    slot_of: Dict[Tuple[str, int], int] = {}

    def slot(ref):
        if ref not in slot_of:
            slot_of[ref] = len(slot_of)
        return slot_of[ref]

    feed_slots = [slot(r) for r in feed_refs]
    feed_dtypes = []
    for n, _ in feed_refs:
        node = graph.nodes[n]
        feed_dtypes.append(node.attrs.get("dtype") if node.op == "Placeholder" else None)
    needed: Dict[str, Set[int]] = {}
    for name in order:
        for s, i in graph.nodes[name].inputs:
            needed.setdefault(s, set()).add(i)
    for n, i in fetch_refs:
        needed.setdefault(n, set()).add(i)

    const_slots = []
    steps = []
    for name in order:
        node = graph.nodes[name]
        if name in fed_nodes:
            for i in needed.get(name, ()):
                if (name, i) not in slot_of:
                    raise CompileError(f"output {i} of fed node {name!r} is needed but not fed")
            continue
        if node.op == "Const":
            if node.value is None:
                node.value = [const_value(node)]
            for i in needed.get(name, ()):
                v = node.value[i]
                if isinstance(v, torch.Tensor) and device.type != "cpu" and _device_resident(v):
                    v = to_device(v, device)
                    node.value[i] = v
                const_slots.append((slot((name, i)), v))
            continue
        if node.op in ("VariableV2", "Variable", "VarHandleOp"):
            raise CompileError(f"variable {name!r} has no value in the checkpoint")
        fn = O.OPS.get(node.op)
        if fn is None:
            raise CompileError(f"op {node.op!r} (node {name!r}) is not supported")
        in_slots = [slot(r) for r in node.inputs]
        outs = needed.get(name, set())
        n_out = (max(outs) + 1) if outs else 0
        out_slots = [slot((name, i)) if i in outs else -1 for i in range(n_out)]
        steps.append((fn, node, in_slots, out_slots))
    fetch_slots = [slot(r) for r in fetch_refs]
    return Program(steps, len(slot_of), feed_slots, fetch_slots, const_slots, device, feed_dtypes,
                   graph, order)


def _device_resident(v: torch.Tensor) -> bool:
    """Shape-like int tensors stay on the host; everything else goes to the device."""
    if v.is_floating_point():
        return True
    return v.numel() > 64
