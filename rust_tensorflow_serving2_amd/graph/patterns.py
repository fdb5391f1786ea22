"""Subgraph pattern matchers for encoder (BERT-style) graphs.

* decomposed LayerNorm (``tf.contrib.layers.layer_norm`` / BERT ``modeling.py``)::

      mean = Mean(x, -1, keep);  var = Mean(SquaredDifference(x, StopGradient(mean)), -1, keep)
      M = Mul(Rsqrt(AddV2(var, eps)), gamma)
      y = AddV2(Mul(x, M), Sub(beta, Mul(mean, M)))          => _LayerNorm(x)

* GELU, tanh form (BERT) and erf form (Keras/TF2)    => activation of _FusedMatMul
* self-attention core::

      q|k|v = Transpose(Reshape(BiasAdd(MatMul(x, Wq|k|v)), [-1,S,H,D]), [0,2,1,3])
      p = Softmax(AddV2(Mul(BatchMatMul(q, k, adj_y), scale), mask_adder))
      y = Reshape(Transpose(BatchMatMul(p, v), [0,2,1,3]), [-1, H*D])
        => _FusedQKV(x)  (one GEMM, concatenated weights)  ->  _Attention(qkv, mask_adder)

Matching is strict: every interior node must be consumed only inside the
pattern; anything else is left to the reference ops.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Set, Tuple

import torch
import torch.nn.functional as F

from . import ops as O
from .placement import to_device
from .ir import Graph, Node

BF16 = torch.bfloat16


# ------------------------------------------------------------------ helpers
def _node(g: Graph, ref) -> Optional[Node]:
    return g.nodes.get(ref[0]) if ref[1] == 0 else None


def _const_t(g: Graph, ref) -> Optional[torch.Tensor]:
    n = g.nodes.get(ref[0])
    if n is None or n.op != "Const" or n.value is None:
        return None
    v = n.value[ref[1]]
    return v if isinstance(v, torch.Tensor) else None


def _scalar(g: Graph, ref) -> Optional[float]:
    v = _const_t(g, ref)
    if v is None or v.numel() != 1:
        return None
    return float(v.reshape(-1)[0])


def _other(n: Node, ref) -> Optional[tuple]:
    if len(n.inputs) != 2:
        return None
    if n.inputs[0] == ref:
        return n.inputs[1]
    if n.inputs[1] == ref:
        return n.inputs[0]
    return None


def _close(a: Optional[float], b: float, tol: float = 1e-4) -> bool:
    return a is not None and abs(a - b) <= tol * max(1.0, abs(b))


def _interior_ok(c, interior: Sequence[Node], out: Node) -> bool:
    names = {n.name for n in interior} | {out.name}
    for n in interior:
        if n.name in c.fetch_nodes:
            return False
        for cname, _p, _i in c.cons.get(n.name, []):
            if cname not in names:
                return False
    return True


def _consumers(c, name: str) -> List[Node]:
    return [c.g.nodes[cn] for cn, _p, _i in c.cons.get(name, [])]


def _remove(g: Graph, nodes: Sequence[Node]):
    for n in nodes:
        g.nodes.pop(n.name, None)


def _axes_last(g, ref, rank_hint=None) -> bool:
    v = _const_t(g, ref)
    if v is None or v.numel() != 1:
        return False
    a = int(v.reshape(-1)[0])
    return a == -1 or (rank_hint is not None and a == rank_hint - 1)


# ------------------------------------------------------------------ fused impls
class LayerNormOp:
    def __init__(self, gamma, beta, eps, device, use_hip):
        self.eps = float(eps)
        self.use_hip = use_hip
        self.g = to_device(gamma.float().reshape(-1), device)
        self.b = to_device(beta.float().reshape(-1), device)

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if self.use_hip and x.is_cuda and x.shape[-1] % 8 == 0 and x.shape[-1] == self.g.numel():
            from ..ops import hip
            from .fused import _to_bf16
            return [hip().layernorm(_to_bf16(x).contiguous(), None, self.g, self.b, self.eps)]
        y = F.layer_norm(x.float(), (x.shape[-1],), self.g.to(x.device), self.b.to(x.device), self.eps)
        return [y if not x.is_cuda else y.to(x.dtype)]


MAX_ATTENTION_SEQ = 4096      # kernels/launch.h kMaxAttentionSeq


class AttentionOp:
    def __init__(self, heads: int, head_dim: int, seq: int, scale: float, use_hip: bool):
        self.h, self.d, self.s, self.scale, self.use_hip = heads, head_dim, seq, scale, use_hip

    def __call__(self, ctx, node, ins):
        qkv = O.to_torch(ins[0])
        adder = O.to_torch(ins[1]) if len(ins) > 1 else None
        S, H, D = self.s, self.h, self.d
        B = qkv.numel() // (S * 3 * H * D)
        if adder is not None:
            if adder.dim() != 4 or adder.shape[1] != 1 or adder.shape[-1] != S:
                raise O.Unsupported("attention mask must be [B|1, 1, S|1, S]")
        if self.use_hip and qkv.is_cuda and D == 64 and 1 <= S <= MAX_ATTENTION_SEQ:
            from ..ops import hip
            from .fused import _to_bf16
            q3 = _to_bf16(qkv).reshape(B, S, 3 * H * D).contiguous()
            mask = None
            bstride = qstride = 0
            if adder is not None:
                mask = adder.float().contiguous().to(qkv.device)
                bstride = S * adder.shape[2] if adder.shape[0] == B and B > 1 else 0
                qstride = S if adder.shape[2] == S else 0
            y = hip().attention(q3, mask, H, self.scale, None, bstride, qstride)
            return [y.reshape(B * S, H * D)]
        q, k, v = qkv.float().reshape(B, S, 3, H, D).permute(2, 0, 3, 1, 4)
        sc = q @ k.transpose(-1, -2) * self.scale
        if adder is not None:
            sc = sc + adder.float().to(sc.device)
        y = (torch.softmax(sc, -1) @ v).permute(0, 2, 1, 3).reshape(B * S, H * D)
        return [y if not qkv.is_cuda else y.to(qkv.dtype)]


# ------------------------------------------------------------------ GELU
def match_gelu_subgraph(g: Graph, c, src: str):
    x = (src, 0)
    cons = _consumers(c, src)
    if src in c.fetch_nodes:
        return None
    # tanh form
    pows = [n for n in cons if n.op == "Pow" and n.inputs[0] == x and _close(_scalar(g, n.inputs[1]), 3.0)]
    if pows:
        pw = pows[0]
        chain = [pw]
        nx = _consumers(c, pw.name)
        if len(nx) != 1 or nx[0].op != "Mul" or not _close(_scalar(g, _other(nx[0], (pw.name, 0))), 0.044715):
            return None
        m = nx[0]
        chain.append(m)
        nx = _consumers(c, m.name)
        if len(nx) != 1 or nx[0].op not in ("Add", "AddV2") or _other(nx[0], (m.name, 0)) != x:
            return None
        a = nx[0]
        chain.append(a)
        nx = _consumers(c, a.name)
        if len(nx) != 1 or nx[0].op != "Mul" or not _close(_scalar(g, _other(nx[0], (a.name, 0))),
                                                          math.sqrt(2 / math.pi)):
            return None
        m1 = nx[0]
        chain.append(m1)
        nx = _consumers(c, m1.name)
        if len(nx) != 1 or nx[0].op != "Tanh":
            return None
        t = nx[0]
        chain.append(t)
        tail = _gelu_tail(g, c, t, x, chain)
        if tail is None:
            return None
        return ("gelu_tanh",) + tail
    # erf form: Erf(x * 1/sqrt2) or Erf(x / sqrt2)
    for n in cons:
        if n.op == "Mul" and _close(_scalar(g, _other(n, x) or ("", 0)), 1 / math.sqrt(2)) or \
                n.op == "RealDiv" and n.inputs[0] == x and _close(_scalar(g, n.inputs[1]), math.sqrt(2)):
            nx = _consumers(c, n.name)
            if len(nx) == 1 and nx[0].op == "Erf":
                tail = _gelu_tail(g, c, nx[0], x, [n, nx[0]])
                if tail is not None:
                    return ("gelu_erf",) + tail
    return None


def _gelu_tail(g, c, t: Node, x, chain: List[Node]):
    """... t -> AddV2(1, t) -> [Mul(0.5, .) -> Mul(x, .)] | [Mul(., Mul(x, 0.5))]"""
    nx = _consumers(c, t.name)
    if len(nx) != 1 or nx[0].op not in ("Add", "AddV2") or not _close(_scalar(g, _other(nx[0], (t.name, 0))), 1.0):
        return None
    a1 = nx[0]
    chain = chain + [a1]
    nx = _consumers(c, a1.name)
    if len(nx) != 1 or nx[0].op != "Mul":
        return None
    m2 = nx[0]
    other = _other(m2, (a1.name, 0))
    if _close(_scalar(g, other), 0.5):            # 0.5 * (1 + t) then * x
        chain.append(m2)
        nx = _consumers(c, m2.name)
        if len(nx) != 1 or nx[0].op != "Mul" or _other(nx[0], (m2.name, 0)) != x:
            return None
        out = nx[0]
    elif other == x:                              # x * (1 + t) then * 0.5
        chain.append(m2)
        nx = _consumers(c, m2.name)
        if len(nx) != 1 or nx[0].op != "Mul" or not _close(_scalar(g, _other(nx[0], (m2.name, 0))), 0.5):
            return None
        out = nx[0]
    else:                                         # (x * 0.5) * (1 + t)
        h = _node(g, other) if other else None
        if h is None or h.op != "Mul" or _other(h, x) is None or not _close(_scalar(g, _other(h, x)), 0.5):
            return None
        chain = chain + [h]
        out = m2
    if not _interior_ok(c, chain, out):
        return None
    # every consumer of x must be inside the pattern (x is the GEMM output being fused)
    names = {n.name for n in chain} | {out.name}
    if any(n.name not in names for n in _consumers(c, x[0])):
        return None
    return chain, out


# ------------------------------------------------------------------ LayerNorm
def fuse_layernorm(g, order, fed, fetch_refs, device, opts):
    from .fused import _Ctx
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        n = g.nodes.get(name)
        if n is None or n.op not in ("Add", "AddV2") or len(n.inputs) != 2:
            continue
        m = _match_ln(g, c, n)
        if m is None:
            continue
        x_ref, gamma, beta, eps, interior = m
        _remove(g, interior)
        n.op = "_LayerNorm"
        n.inputs = [x_ref]
        n.ctrl = []
        n.attrs = {"_impl": LayerNormOp(gamma, beta, eps, device, c.use_hip)}
        c.refresh()


def _match_ln(g, c, out: Node):
    for ia, ib in ((0, 1), (1, 0)):
        mul1, sub = _node(g, out.inputs[ia]), _node(g, out.inputs[ib])
        if mul1 is None or sub is None or mul1.op != "Mul" or sub.op != "Sub":
            continue
        beta = _const_t(g, sub.inputs[0])
        mul2 = _node(g, sub.inputs[1])
        if beta is None or mul2 is None or mul2.op != "Mul":
            continue
        for jx in (0, 1):
            x_ref = mul1.inputs[jx]
            M = _node(g, mul1.inputs[1 - jx])
            if M is None or M.op != "Mul":
                continue
            mean_ref = _other(mul2, (M.name, 0))
            mean = _node(g, mean_ref) if mean_ref else None
            if mean is None or mean.op != "Mean" or mean.inputs[0] != x_ref or not _axes_last(g, mean.inputs[1]):
                continue
            rs = gamma = None
            for k in (0, 1):
                a, b = _node(g, M.inputs[k]), _const_t(g, M.inputs[1 - k])
                if a is not None and a.op == "Rsqrt" and b is not None:
                    rs, gamma = a, b
            if rs is None:
                continue
            add = _node(g, rs.inputs[0])
            if add is None or add.op not in ("Add", "AddV2"):
                continue
            var = eps = None
            for k in (0, 1):
                a, e = _node(g, add.inputs[k]), _scalar(g, add.inputs[1 - k])
                if a is not None and a.op == "Mean" and e is not None:
                    var, eps = a, e
            if var is None or not _axes_last(g, var.inputs[1]):
                continue
            sqd = _node(g, var.inputs[0])
            if sqd is None or sqd.op != "SquaredDifference" or sqd.inputs[0] != x_ref:
                continue
            mref = sqd.inputs[1]
            sg = _node(g, mref)
            interior = [mul1, sub, mul2, M, mean, rs, add, var, sqd]
            if sg is not None and sg.op in ("StopGradient", "Identity"):
                if sg.inputs[0] != (mean.name, 0):
                    continue
                interior.append(sg)
            elif mref != (mean.name, 0):
                continue
            if not _interior_ok(c, interior, out):
                continue
            return x_ref, gamma, beta, eps, interior
    return None


# ------------------------------------------------------------------ attention
def _dense_src(g, c, ref):
    """ref = BiasAdd(MatMul(x, W), b) (or MatMul alone) -> (x, W[K,N], b, nodes)."""
    n = _node(g, ref)
    nodes = []
    bias = None
    if n is not None and n.op in ("BiasAdd", "Add", "AddV2"):
        b = _const_t(g, n.inputs[1])
        if b is None:
            return None
        bias = b.float().reshape(-1)
        nodes.append(n)
        n = _node(g, n.inputs[0])
    if n is None or n.op != "MatMul" or n.attr("transpose_a", False):
        return None
    w = _const_t(g, n.inputs[1])
    if w is None:
        return None
    w = w.float()
    if n.attr("transpose_b", False):
        w = w.t()
    nodes.append(n)
    if bias is None:
        bias = torch.zeros(w.shape[1], device=w.device)
    return n.inputs[0], w, bias, nodes


def _heads_of(g, c, ref, S_expected=None):
    """ref = Transpose(Reshape(dense, [-1,S,H,D]), [0,2,1,3]) -> (dense ref, S, H, D, nodes)."""
    t = _node(g, ref)
    if t is None or t.op != "Transpose":
        return None
    perm = _const_t(g, t.inputs[1])
    if perm is None or perm.reshape(-1).tolist() != [0, 2, 1, 3]:
        return None
    r = _node(g, t.inputs[0])
    if r is None or r.op != "Reshape":
        return None
    shp = _const_t(g, r.inputs[1])
    if shp is None or shp.numel() != 4:
        return None
    _b, S, H, D = [int(v) for v in shp.reshape(-1).tolist()]
    if S <= 0 or H <= 0 or D <= 0:
        return None
    return r.inputs[0], S, H, D, [t, r]


def fuse_attention(g, order, fed, fetch_refs, device, opts):
    from .fused import FusedMatMul, _Ctx
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in list(order):
        out = g.nodes.get(name)
        if out is None or out.op != "Reshape":
            continue
        t2 = _node(g, out.inputs[0])
        if t2 is None or t2.op != "Transpose":
            continue
        perm = _const_t(g, t2.inputs[1])
        if perm is None or perm.reshape(-1).tolist() != [0, 2, 1, 3]:
            continue
        pv = _node(g, t2.inputs[0])
        if pv is None or pv.op not in ("BatchMatMul", "BatchMatMulV2", "BatchMatMulV3") or \
                pv.attr("adj_x", False) or pv.attr("adj_y", False):
            continue
        sm = _node(g, pv.inputs[0])
        if sm is None or sm.op != "Softmax":
            continue
        cur = _node(g, sm.inputs[0])
        adder_ref = None
        scale = 1.0
        interior = [t2, pv, sm]
        if cur is not None and cur.op in ("Add", "AddV2"):
            # scores + adder (either order): scores side is the Mul/BatchMatMul
            a0, a1 = _node(g, cur.inputs[0]), _node(g, cur.inputs[1])
            if a0 is not None and a0.op in ("Mul", "BatchMatMul", "BatchMatMulV2", "BatchMatMulV3"):
                adder_ref, cur2 = cur.inputs[1], a0
            else:
                adder_ref, cur2 = cur.inputs[0], a1
            interior.append(cur)
            cur = cur2
        if cur is not None and cur.op == "Mul":
            sv = None
            for k in (0, 1):
                s = _scalar(g, cur.inputs[k])
                if s is not None:
                    sv, nxt = s, _node(g, cur.inputs[1 - k])
            if sv is None:
                continue
            scale = sv
            interior.append(cur)
            cur = nxt
        qk = cur
        if qk is None or qk.op not in ("BatchMatMul", "BatchMatMulV2", "BatchMatMulV3") or \
                qk.attr("adj_x", False) or not qk.attr("adj_y", False):
            continue
        interior.append(qk)
        hq, hk, hv = _heads_of(g, c, qk.inputs[0]), _heads_of(g, c, qk.inputs[1]), _heads_of(g, c, pv.inputs[1])
        if hq is None or hk is None or hv is None:
            continue
        S, H, D = hq[1], hq[2], hq[3]
        if (hk[1], hk[2], hk[3]) != (S, H, D) or (hv[1], hv[2], hv[3]) != (S, H, D):
            continue
        fshape = _const_t(g, out.inputs[1])
        if fshape is None or fshape.reshape(-1).tolist()[-1] != H * D:
            continue
        dq, dk, dv = _dense_src(g, c, hq[0]), _dense_src(g, c, hk[0]), _dense_src(g, c, hv[0])
        interior += hq[4] + hk[4] + hv[4]
        if dq and dk and dv and dq[0] == dk[0] == dv[0]:
            qkv_nodes = dq[3] + dk[3] + dv[3]
            if not _interior_ok(c, interior + qkv_nodes, out):
                continue
            w = torch.cat([dq[1], dk[1], dv[1]], dim=1)
            b = torch.cat([dq[2], dk[2], dv[2]])
            qkv_name = g.unique_name(out.name + "/fused_qkv")
            qkv = Node(name=qkv_name, op="_FusedQKV", inputs=[dq[0]],
                       attrs={"_impl": FusedMatMul(w, b, "none", False, device, c.use_hip, qkv_name)})
            g.add(qkv)
            _remove(g, interior + qkv_nodes)
            out.op = "_Attention"
            out.inputs = [(qkv_name, 0)] + ([adder_ref] if adder_ref is not None else [])
            out.ctrl = []
            out.attrs = {"_impl": AttentionOp(H, D, S, scale, c.use_hip)}
        else:
            # projections not fusable into one GEMM: keep them, concatenate outputs at run time
            continue
        c.refresh()


# ------------------------------------------------------------------ embeddings
class EmbeddingLNOp:
    """LN(sum of row gathers + position rows), the BERT embedding block
    (modeling.py ``embedding_lookup`` / ``embedding_postprocessor``) as one
    ``embed_ln`` launch: one wave per token, tables held in bf16."""

    def __init__(self, tables, pos, seq, gamma, beta, eps, device, use_hip):
        self.seq, self.eps, self.use_hip = int(seq), float(eps), use_hip
        self.tables_f = [t.float().contiguous() for t in tables]
        self.pos_f = None if pos is None else pos.float().reshape(-1, tables[0].shape[1]).contiguous()
        self.g = to_device(gamma.float().reshape(-1), device)
        self.b = to_device(beta.float().reshape(-1), device)
        self.hip_ok = use_hip and device.type == "cuda" and len(tables) <= 2
        if self.hip_ok:
            self.tables = [to_device(t, device, BF16) for t in tables]
            self.pos = None if pos is None else to_device(self.pos_f, device, BF16)
            self.tables_f = self.pos_f = None     # only the bf16 copies stay resident
        else:
            self.tables_f = [to_device(t, device) for t in self.tables_f]
            self.pos_f = None if self.pos_f is None else to_device(self.pos_f, device)

    def __call__(self, ctx, node, ins):
        idx = [O.to_torch(v) for v in ins]
        S = self.seq
        n = idx[0].numel()
        for i in idx[1:]:
            if i.numel() != n:
                raise O.OpError(f"{node.name}: embedding index counts differ")
        if n % S:
            raise O.OpError(f"{node.name}: {n} ids do not reshape to [-1, {S}]")
        if self.hip_ok:
            from ..ops import hip
            dev = self.g.device
            ii = [i.to(dev, torch.int32).reshape(-1).contiguous() for i in idx]
            y = hip().embed_ln(ii[0], ii[1] if len(ii) > 1 else None, self.tables[0], self.pos,
                               self.tables[1] if len(ii) > 1 else None, self.g, self.b, self.eps, S)
            return [y.reshape(-1, S, y.shape[-1])]
        acc = None
        for i, t in zip(idx, self.tables_f):
            i = i.reshape(-1).to(t.device).long()
            if t.device.type == "cpu":
                if n and (int(i.min()) < 0 or int(i.max()) >= t.shape[0]):
                    raise O.OpError(f"{node.name}: indices out of range [0, {t.shape[0]})")
                r = t.index_select(0, i)
            else:
                ok = (i >= 0) & (i < t.shape[0])
                r = t.index_select(0, i.clamp(0, t.shape[0] - 1)) * ok[:, None].float()
            acc = r if acc is None else acc + r
        y = acc.reshape(-1, S, acc.shape[-1])
        if self.pos_f is not None:
            y = y + self.pos_f[:S]
        return [F.layer_norm(y, (y.shape[-1],), self.g, self.b, self.eps)]


def _gather_term(g, c, ref):
    """Reshape(GatherV2(table, idx, 0), [-1, S, Hd]) -> (table, idx_ref, S, nodes)."""
    rs = _node(g, ref)
    if rs is None or rs.op != "Reshape":
        return None
    shp = _const_t(g, rs.inputs[1])
    ga = _node(g, rs.inputs[0])
    if shp is None or ga is None or ga.op != "GatherV2" or int(ga.attr("batch_dims", 0)) != 0:
        return None
    shp = shp.reshape(-1).tolist()
    table, ax = _const_t(g, ga.inputs[0]), _scalar(g, ga.inputs[2])
    if table is None or table.dim() != 2 or ax != 0 or len(shp) != 3 or shp[0] != -1 or shp[2] != table.shape[1]:
        return None
    return table, ga.inputs[1], int(shp[1]), [rs, ga]


def fuse_embedding(g, order, fed, fetch_refs, device, opts):
    """_LayerNorm(word gather + [type gather] + [position rows]) -> _EmbeddingLN."""
    from .fused import _Ctx
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        ln = g.nodes.get(name)
        if ln is None or ln.op != "_LayerNorm":
            continue
        leaves, interior, stack = [], [], [ln.inputs[0]]
        while stack and len(leaves) <= 3:
            ref = stack.pop()
            n = _node(g, ref)
            if n is not None and n.op in ("Add", "AddV2") and len(n.inputs) == 2:
                interior.append(n)
                stack += n.inputs
            else:
                leaves.append(ref)
        if not interior or len(leaves) > 3:
            continue
        gathers, pos = [], []
        for ref in leaves:
            gt = _gather_term(g, c, ref)
            if gt is not None:
                gathers.append(gt)
                continue
            v = _const_t(g, ref)
            if v is None:
                break
            pos.append(v)
        else:
            if not gathers or len(pos) > 1:
                continue
            S, Hd = gathers[0][2], gathers[0][0].shape[1]
            if any(gt[2] != S or gt[0].shape[1] != Hd for gt in gathers):
                continue
            p = pos[0] if pos else None
            if p is not None and tuple(p.shape) not in ((1, S, Hd), (S, Hd)):
                continue
            impl = ln.attrs["_impl"]
            nodes = interior + [n for gt in gathers for n in gt[3]]
            if not _interior_ok(c, nodes, ln):
                continue
            gathers.sort(key=lambda gt: -gt[0].shape[0])    # largest (word) table first
            _remove(g, nodes)
            ln.op = "_EmbeddingLN"
            ln.inputs = [gt[1] for gt in gathers]
            ln.ctrl = []
            ln.attrs = {"_impl": EmbeddingLNOp([gt[0] for gt in gathers], p, S, impl.g, impl.b, impl.eps,
                                               device, c.use_hip)}
            c.refresh()


# ------------------------------------------------------------------ attention mask
class KeyMaskAdderOp:
    """(one - X) * scale for a key mask X [B, 1, S], shaped [B, 1, 1, S]: the
    BERT attention adder (modeling.py ``create_attention_mask_from_input_mask``
    + ``(1 - mask) * -10000``) without materialising the [B, S, S] broadcast.
    Only _Attention consumes it, and it broadcasts over the query axis."""

    def __init__(self, one, scale):
        self.one, self.scale = float(one), float(scale)

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if x.dim() != 3 or x.shape[1] != 1:
            raise O.Unsupported("key mask must be [B, 1, S]")
        if x.is_cuda and x.dtype in (torch.int32, torch.float32):
            from ..ops import hip
            return [hip().key_mask_adder(x.contiguous(), self.one, self.scale).unsqueeze(1)]   # one launch
        return [(x.float() * -self.scale).add_(self.one * self.scale).unsqueeze(1)]


def fuse_key_mask(g, order, fed, fetch_refs, device, opts):
    """Mul(Sub(1, ExpandDims(Mul(ones[1,S,1], X), 1)), c) feeding only _Attention
    nodes -> _KeyMaskAdder(X)."""
    from .fused import _Ctx
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        mul = g.nodes.get(name)
        if mul is None or mul.op != "Mul" or len(mul.inputs) != 2 or name in c.fetch_nodes:
            continue
        cons = c.cons.get(name, [])
        if not cons or any(g.nodes[cn].op != "_Attention" or pos != 1 or oi != 0 for cn, pos, oi in cons):
            continue
        for k in (0, 1):
            sub, scale = _node(g, mul.inputs[k]), _scalar(g, mul.inputs[1 - k])
            if sub is not None and sub.op == "Sub" and scale is not None:
                break
        else:
            continue
        one, ex = _scalar(g, sub.inputs[0]), _node(g, sub.inputs[1])
        if one is None or ex is None or ex.op != "ExpandDims" or _scalar(g, ex.inputs[1]) != 1:
            continue
        bm = _node(g, ex.inputs[0])
        if bm is None or bm.op != "Mul" or len(bm.inputs) != 2:
            continue
        x_ref = None
        for k in (0, 1):
            ones = _const_t(g, bm.inputs[k])
            if ones is not None and ones.dim() == 3 and ones.shape[0] == 1 and ones.shape[2] == 1 and \
                    bool((ones == 1).all()):
                x_ref = bm.inputs[1 - k]
                S = ones.shape[1]
        if x_ref is None or not _interior_ok(c, [sub, ex, bm], mul):
            continue
        interior = [sub, ex, bm]
        cast = _node(g, x_ref)
        if cast is not None and cast.op == "Cast" and not cast.ctrl and \
                O.dt_attr(cast, "DstT") == torch.float32 and _interior_ok(c, interior + [cast], mul):
            interior.append(cast)        # the op casts to f32 itself
            x_ref = cast.inputs[0]
        _remove(g, interior)
        mul.op = "_KeyMaskAdder"
        mul.inputs = [x_ref]
        mul.ctrl = []
        mul.attrs = {"_impl": KeyMaskAdderOp(one, scale), "_seq": S}
        c.refresh()


def bert_passes():
    return [fuse_layernorm, fuse_embedding, fuse_attention, fuse_key_mask]


def late_passes():
    """Passes over the fused graph (after every GEMM is a _FusedMatMul).  None
    here; the LayerNorm fold runs last (graph/fused.py defer_layernorm: round
    3's fold spilled registers in the 8-wave tiles and was removed in round 4,
    profiles/round3/ln_fold.md; round 5's epilogue reads its per-column
    vectors from LDS instead)."""
    return []
