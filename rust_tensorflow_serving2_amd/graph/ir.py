"""Graph IR: a GraphDef parsed into plain Python nodes that passes can rewrite.

Tensor references follow TF's text form: ``"node"`` == ``"node:0"``,
``"node:k"`` is output k, ``"^node"`` is a control dependency.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

from ..schema import tf


def parse_ref(ref: str) -> Tuple[str, int]:
    if ref.startswith("^"):
        return ref[1:], -1
    if ":" in ref:
        n, i = ref.rsplit(":", 1)
        if i.isdigit():
            return n, int(i)
    return ref, 0


def fmt_ref(node: str, idx: int) -> str:
    return node if idx == 0 else f"{node}:{idx}"


def attr_to_py(a):
    kind = a.WhichOneof("value")
    if kind is None:
        return None
    if kind == "list":
        lv = a.list
        for fld in ("s", "i", "f", "b", "type", "shape", "tensor", "func"):
            vals = getattr(lv, fld)
            if len(vals):
                if fld == "shape":
                    return [tuple(d.size for d in s.dim) for s in vals]
                if fld == "tensor":
                    from .. import native
                    return [native.decode_tensor_proto(t.SerializeToString()) for t in vals]
                if fld == "s":
                    return [bytes(x) for x in vals]
                return list(vals)
        return []
    v = getattr(a, kind)
    if kind == "shape":
        if v.unknown_rank:
            return None
        return tuple(d.size for d in v.dim)
    if kind == "tensor":
        from .. import native
        return native.decode_tensor_proto(v.SerializeToString())
    if kind == "s":
        return bytes(v)
    if kind == "func":
        return v.name
    return v


@dataclass
class Node:
    name: str
    op: str
    inputs: List[Tuple[str, int]] = field(default_factory=list)
    ctrl: List[str] = field(default_factory=list)
    attrs: Dict[str, object] = field(default_factory=dict)
    device: str = ""
    # populated by passes: constant value(s) of the outputs
    value: Optional[list] = None

    def attr(self, k, default=None):
        v = self.attrs.get(k, default)
        return default if v is None else v

    def sattr(self, k, default="") -> str:
        v = self.attrs.get(k)
        if v is None:
            return default
        return v.decode() if isinstance(v, bytes) else v


class Graph:
    def __init__(self):
        self.nodes: Dict[str, Node] = {}
        self.order: List[str] = []
        self.functions: Dict[str, object] = {}

    def add(self, node: Node) -> Node:
        if node.name in self.nodes:
            raise ValueError(f"duplicate node name {node.name}")
        self.nodes[node.name] = node
        self.order.append(node.name)
        return node

    def unique_name(self, base: str) -> str:
        name, i = base, 0
        while name in self.nodes:
            i += 1
            name = f"{base}_{i}"
        return name

    def consumers(self) -> Dict[str, List[Tuple[str, int, int]]]:
        """producer -> [(consumer, input_pos, output_idx)]"""
        out: Dict[str, List[Tuple[str, int, int]]] = {}
        for n in self.nodes.values():
            for pos, (src, idx) in enumerate(n.inputs):
                out.setdefault(src, []).append((n.name, pos, idx))
        return out

    def topo(self, targets: Iterable[str], stop: Set[str] = frozenset()) -> List[str]:
        """Nodes needed to compute ``targets`` (control deps included), producers
        first.  Nodes in ``stop`` are treated as leaves (fed tensors)."""
        order: List[str] = []
        state: Dict[str, int] = {}
        for t in targets:
            if t not in self.nodes:
                raise KeyError(f"node {t!r} not in graph")
            stack = [(t, False)]
            while stack:
                n, done = stack.pop()
                if done:
                    if state.get(n) != 2:
                        state[n] = 2
                        order.append(n)
                    continue
                st = state.get(n)
                if st == 2:
                    continue
                if st == 1:
                    continue
                state[n] = 1
                stack.append((n, True))
                if n in stop:
                    continue
                node = self.nodes[n]
                deps = [s for s, _ in node.inputs] + list(node.ctrl)
                for d in reversed(deps):
                    if d not in self.nodes:
                        raise KeyError(f"{n}: input {d!r} not in graph")
                    if state.get(d) is None:
                        stack.append((d, False))
                    elif state.get(d) == 1 and d not in stop:
                        raise ValueError(f"cycle in graph at {d}")
        return order


def from_graph_def(gd) -> Graph:
    g = Graph()
    for nd in gd.node:
        node = Node(name=nd.name, op=nd.op, device=nd.device)
        for ref in nd.input:
            n, i = parse_ref(ref)
            if i < 0:
                node.ctrl.append(n)
            else:
                node.inputs.append((n, i))
        for k, v in nd.attr.items():
            node.attrs[k] = attr_to_py(v)
        g.add(node)
    for fn in gd.library.function:
        g.functions[fn.signature.name] = fn
    inline_functions(g)
    return g


# ---------------------------------------------------------------- TF2 function inlining
# Output-argument layout of builtin multi-output ops, for resolving function-body
# tensor names "node:out_arg:idx" to flat output indices.
_OUT_ARGS = {
    "FusedBatchNorm": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2"],
    "FusedBatchNormV2": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2"],
    "FusedBatchNormV3": ["y", "batch_mean", "batch_variance", "reserve_space_1", "reserve_space_2",
                         "reserve_space_3"],
    "TopKV2": ["values", "indices"],
    "Unique": ["y", "idx"],
    "BroadcastGradientArgs": ["r0", "r1"],
}
CALL_OPS = ("PartitionedCall", "StatefulPartitionedCall")


def _body_ref(ref: str, local: Dict[str, str], args: Dict[str, Tuple[str, int]],
              out_base: Dict[str, Tuple[str, Dict[str, int]]]) -> Tuple[str, int]:
    """Function-body tensor name -> (graph node, output index)."""
    if ref in args:
        return args[ref]
    parts = ref.split(":")
    node = parts[0]
    if node not in local:
        raise ValueError(f"function body references unknown tensor {ref!r}")
    if len(parts) == 1:
        return local[node], 0
    if len(parts) == 2:                       # "node:idx" (GraphDef style, rare in bodies)
        return local[node], int(parts[1])
    out_arg, idx = parts[1], int(parts[2])
    op, offsets = out_base[node]
    if out_arg in offsets:
        return local[node], offsets[out_arg] + idx
    return local[node], idx                   # single (list) output argument


def inline_functions(g: Graph, max_depth: int = 64) -> int:
    """Inline every PartitionedCall / StatefulPartitionedCall (and direct calls of
    library functions) so TF2 SavedModels become one flat graph the compiler
    can fold and fuse.  The call node becomes an IdentityN of the function's
    return tensors, so its consumers and control dependents are untouched.
    Returns the number of calls inlined."""
    if not g.functions:
        return 0
    done = 0
    for _round in range(max_depth):
        calls = [n for n in list(g.nodes.values())
                 if (n.op in CALL_OPS and n.attrs.get("f")) or n.op in g.functions]
        if not calls:
            return done
        for call in calls:
            fname = call.attrs.get("f") if call.op in CALL_OPS else call.op
            fdef = g.functions.get(fname)
            if fdef is None:
                raise ValueError(f"{call.name}: function {fname!r} not in the graph's library")
            sig = fdef.signature
            if len(sig.input_arg) != len(call.inputs):
                raise ValueError(f"{call.name}: {len(call.inputs)} inputs for {fname} "
                                 f"which takes {len(sig.input_arg)}")
            args = {a.name: src for a, src in zip(sig.input_arg, call.inputs)}
            local: Dict[str, str] = {}
            out_base: Dict[str, Tuple[str, Dict[str, int]]] = {}
            for nd in fdef.node_def:
                local[nd.name] = g.unique_name(f"{call.name}/{nd.name}")
                offsets: Dict[str, int] = {}
                # (Stateful)PartitionedCall has ONE list output arg ("output"); a direct
                # call of a library function exposes that function's output args
                inner = g.functions.get(nd.op)
                names = [a.name for a in inner.signature.output_arg] if inner is not None \
                    else _OUT_ARGS.get(nd.op, [])
                for k, a in enumerate(names):
                    offsets[a] = k
                out_base[nd.name] = (nd.op, offsets)
            for nd in fdef.node_def:
                node = Node(name=local[nd.name], op=nd.op, device=nd.device)
                for ref in nd.input:
                    if ref.startswith("^"):
                        c = ref[1:]
                        if c in local:
                            node.ctrl.append(local[c])
                        elif c in args:
                            node.ctrl.append(args[c][0])
                        continue
                    node.inputs.append(_body_ref(ref, local, args, out_base))
                for k, v in nd.attr.items():
                    node.attrs[k] = attr_to_py(v)
                node.ctrl.extend(call.ctrl)
                g.add(node)
            rets = [_body_ref(fdef.ret[a.name], local, args, out_base) for a in sig.output_arg]
            call.op = "IdentityN"
            call.inputs = rets
            call.attrs = {"T": [0] * len(rets), "_inlined": fname}
            # keep the call's control inputs only through the inlined nodes
            call.ctrl = [local[n] for n in fdef.control_ret.values() if n in local]
            done += 1
    raise ValueError("function call nesting deeper than %d" % max_depth)


def restore_keys(g: Graph) -> Dict[str, str]:
    """Variable node -> checkpoint key, read off the saver's restore subgraph
    (RestoreV2 tensor_names -> [Identity] -> Assign / AssignVariableOp).  TF2
    SavedModels key variables by object path ("layer/kernel/.ATTRIBUTES/
    VARIABLE_VALUE"), which neither the node name nor shared_name carries."""
    def through_identity(name: str, idx: int) -> Tuple[str, int]:
        seen = 0
        while name in g.nodes and g.nodes[name].op in ("Identity", "IdentityN") and seen < 64:
            n = g.nodes[name]
            name, idx = n.inputs[idx if n.op == "IdentityN" else 0]
            seen += 1
        return name, idx

    out: Dict[str, str] = {}
    for n in g.nodes.values():
        if n.op not in ("Assign", "AssignVariableOp") or len(n.inputs) < 2:
            continue
        var, _ = through_identity(*n.inputs[0])
        src, idx = through_identity(*n.inputs[1])
        r = g.nodes.get(src)
        if r is None or r.op not in ("RestoreV2", "Restore", "RestoreSlice") or len(r.inputs) < 2:
            continue
        names_node = g.nodes.get(r.inputs[1][0])
        if names_node is None or names_node.op != "Const":
            continue
        vals = np.asarray(names_node.attrs.get("value"), dtype=object).reshape(-1)
        if idx < len(vals):
            key = vals[idx]
            out[var] = key.decode() if isinstance(key, bytes) else str(key)
    return out
