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
    return g
