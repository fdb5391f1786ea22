"""Fusion passes: rewrite TF op chains into fused ops backed by gfx950 kernels.

Patterns (matched on the constant-folded IR, only when every intermediate has
a single consumer and is not fetched):

* ``[Pad] -> Conv2D -> [BiasAdd] -> [FusedBatchNorm*] -> [Add(residual)] -> [Relu]``
  => ``_FusedConv2D``: BN folded into the weights at load time (w' = w*gamma/
  sqrt(var+eps), b' = beta - mean*scale), spatial Pad absorbed into the conv's
  explicit padding, residual add + ReLU in the MFMA kernel's epilogue.  A conv
  whose input has C % 8 != 0 (the RGB stem) reads the fp32 request tensor
  directly (ingest cast fused into the operand loads).
* ``MatMul -> [BiasAdd] -> [Add(residual)] -> [Relu|Tanh|GELU]`` => ``_FusedMatMul``
  (fp32 output when it feeds a Softmax/ArgMax head or is fetched).
* ``Mean(NHWC, axes=[1,2])`` => ``_GlobalAvgPool``;  ``MaxPool`` => ``_MaxPool``;
  the ResNet stem ``_FusedConv2D(7x7/2, RGB) -> _MaxPool(3x3/2)`` => ``_StemPool``.
* ``Softmax(x)`` + ``ArgMax(x, -1)`` on the same logits => ``_SoftmaxArgMax``.
* BERT: decomposed LayerNorm => ``_LayerNorm``; tanh/erf GELU subgraphs => act
  of the producing ``_FusedMatMul``; Q/K/V projections + attention core =>
  ``_FusedQKV`` + ``_Attention`` (see ``bert_passes``).

On a CUDA/HIP device the fused ops launch the ``_hip`` kernels (bf16 operands,
fp32 accumulate); on the CPU they run an fp32 torch reference of the *same*
folded parameters, which is how the passes are validated without a GPU.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence, Set, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from ..utils import tensors as T
from . import ops as O
from .ir import Graph, Node
from .placement import to_device, zeros

BF16 = torch.bfloat16


# ------------------------------------------------------------------ helpers
def _const(g: Graph, ref) -> Optional[torch.Tensor]:
    n = g.nodes.get(ref[0])
    if n is None or n.op != "Const" or n.value is None:
        return None
    v = n.value[ref[1]] if ref[1] < len(n.value) else None
    return v if isinstance(v, torch.Tensor) else None


class _Ctx:
    def __init__(self, g: Graph, order: List[str], fed: Set[str], fetch_refs, device, opts):
        self.g = g
        self.order = order
        self.fed = fed
        self.fetch_nodes = {n for n, _ in fetch_refs}
        self.fetch_refs = set(fetch_refs)
        self.device = device
        self.opts = opts
        self.use_hip = device.type == "cuda"
        self.cons = g.consumers()

    def only_consumer(self, name: str, idx: int = 0) -> Optional[Node]:
        """The unique consumer of output ``idx`` of ``name`` (and no other output used)."""
        if name in self.fetch_nodes:
            return None
        cs = self.cons.get(name, [])
        if len(cs) != 1:
            return None
        cname, _pos, oidx = cs[0]
        if oidx != idx:
            return None
        return self.g.nodes[cname]

    def refresh(self):
        self.cons = self.g.consumers()


def _merge_ctrl(nodes: Sequence[Node]) -> List[str]:
    out: List[str] = []
    names = {n.name for n in nodes}
    for n in nodes:
        for c in n.ctrl:
            if c not in out and c not in names:
                out.append(c)
    return out


def _finalize(g: Graph, chain: List[Node], op: str, inputs, attrs) -> Node:
    last = chain[-1]
    ctrl = _merge_ctrl(chain)
    for n in chain[:-1]:
        del g.nodes[n.name]
    last.op = op
    last.inputs = list(inputs)
    last.ctrl = ctrl
    last.attrs = attrs
    last.value = None
    return last


def _pad_k(w_nk: torch.Tensor, mult: int = 64) -> torch.Tensor:
    n, k = w_nk.shape
    kp = -(-k // mult) * mult
    if kp != k:
        w_nk = torch.cat([w_nk, torch.zeros(n, kp - k, dtype=w_nk.dtype, device=w_nk.device)], dim=1)
    return w_nk


def _to_bf16(x: torch.Tensor) -> torch.Tensor:
    if x.dtype == BF16:
        return x
    if x.dtype == torch.float32 and x.is_cuda and x.is_contiguous():
        from ..ops import hip
        return hip().cast_bf16(x)
    return x.to(BF16).contiguous()


# ------------------------------------------------------------------ fused op impls
class FusedConv:
    """Conv2D(+folded BN/bias)(+residual)(+act).  Weights: HWIO fp32 (reference)
    and [Cout][Kpad] bf16 (kernel)."""

    def __init__(self, w_hwio: torch.Tensor, bias: torch.Tensor, strides, padding: str, pads, act: str,
                 device: torch.device, use_hip: bool, name: str):
        self.kh, self.kw, self.cin, self.cout = w_hwio.shape
        self.sh, self.sw = strides
        self.padding = padding          # "SAME" | "VALID" | "EXPLICIT"
        self.pads = pads                # (pt, pb, pl, pr) for EXPLICIT
        self.act = act
        self.use_hip = use_hip
        self.name = name
        self.device = device
        # RGB(A) stems: the fp32 request is re-laid out as zero-bordered bf16 RGBA
        # (ingest_c4_padded), weights as [Cout][kh (padded to even)][8 taps][4 ch]:
        # a 64-deep k-tile is then 2 filter rows x 8 taps x 4 channels = two
        # contiguous 64-B runs of the padded image, DMA'd with no bounds checks
        self.c4 = use_hip and self.cin <= 4 and self.kw <= 8
        self.khp = self.kh + (self.kh % 2) if self.c4 else self.kh
        if use_hip:
            if self.c4:
                w4 = torch.zeros(self.khp, 8, 4, self.cout, device=w_hwio.device)
                w4[:self.kh, :self.kw, :self.cin, :] = w_hwio.float()
                w_nk = w4.permute(3, 0, 1, 2).reshape(self.cout, self.khp * 32)
            else:
                k = self.kh * self.kw * self.cin
                w_nk = w_hwio.permute(3, 0, 1, 2).reshape(self.cout, k)
            self.w = to_device(_pad_k(w_nk).to(BF16), device)
            self.b = to_device(bias.float(), device)
        else:
            self.w_ref = to_device(w_hwio.float(), device)
            self.b_ref = to_device(bias.float(), device)

    # ---- post-activation output (ResNet v2 pre-activation of the next block)
    post = None          # (scale [Cout], shift [Cout], act) on the device / CPU
    post_mode = None     # "dual": [raw, post]; "only": [post]

    def set_post(self, scale: torch.Tensor, shift: torch.Tensor, act: str, mode: str):
        dev = self.device if self.use_hip else (self.w_ref.device if hasattr(self, "w_ref") else "cpu")
        self.post = (to_device(scale.float(), dev), to_device(shift.float(), dev), act)
        self.post_mode = mode

    def post_ok(self) -> bool:
        """The fused kernels write the post output only on the cgemm / halo
        paths (64-aligned channels); the CPU reference always can."""
        return not self.use_hip or (not self.c4 and self.cin % 64 == 0 and self.cout % 8 == 0)

    def pads_for(self, h, w):
        if self.padding == "SAME":
            return O.tf_same_pads(h, self.kh, self.sh) + O.tf_same_pads(w, self.kw, self.sw)
        if self.padding == "EXPLICIT":
            return tuple(self.pads)
        return (0, 0, 0, 0)

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        res = O.to_torch(ins[1]) if len(ins) > 1 else None
        pt, pb, pl, pr = self.pads_for(x.shape[1], x.shape[2])
        if not self.use_hip:
            y = F.conv2d(F.pad(x.float().permute(0, 3, 1, 2), [pl, pr, pt, pb]),
                         self.w_ref.permute(3, 2, 0, 1), stride=(self.sh, self.sw))
            y = y.permute(0, 2, 3, 1) + self.b_ref
            if res is not None:
                y = y + res.float()
            return _with_post(self, _ref_act(y, self.act).contiguous())
        from ..ops import ACT, hip, tuned_config
        if self.c4:
            # fp32 RGB request -> zero-bordered bf16 RGBA sized for the padded
            # (khp x 8) filter; the conv itself then has no padding
            h, w = x.shape[1], x.shape[2]
            ho = (h + pt + pb - self.kh) // self.sh + 1
            wo = (w + pl + pr - self.kw) // self.sw + 1
            hp, wp = (ho - 1) * self.sh + self.khp, (wo - 1) * self.sw + 8
            x = hip().ingest_c4_padded(x.float().contiguous(), hp, wp, pt, pl)
            pt = pb = pl = pr = 0
        elif self.cin % 8 != 0:
            x = x.float().contiguous()            # generic: fp32 operand gather + cast in-kernel
        else:
            x = _to_bf16(x).contiguous()
        if res is not None:
            res = _to_bf16(res).contiguous()
        H = hip()
        n, h, w, _ = x.shape
        kh, kw = (self.khp, 8) if self.c4 else (self.kh, self.kw)
        ho = (h + pt + pb - kh) // self.sh + 1
        wo = (w + pl + pr - kw) // self.sw + 1
        M = n * ho * wo
        args = (x, self.w, self.b, res, kh, kw, self.sh, self.sw, pt, pb, pl, pr, ACT[self.act])
        out = torch.empty((n, ho, wo, self.cout), device=x.device, dtype=BF16)
        key = ("conv", tuple(x.shape), x.dtype, self.cout, kh, kw, self.sh, res is not None, self.act, self.post_mode)
        K = kh * 32 if self.c4 else kh * kw * self.cin
        dma = not self.c4 and self.cin % 8 == 0      # bf16 dense/im2col operands -> DMA-ring configs apply
        # pipelined cgemm kernel applies (im2col / dense with C % 64, or the padded RGBA stem)
        aligned = (dma and self.cin % 64 == 0) or self.c4
        halo = aligned and not self.c4 and kh == 3 and kw == 3 and self.sh == 1 and self.sw == 1
        kw_post, outs = _post_kwargs(self, out)
        run = lambda c, s: H.conv2d(*args, cfg=c, out=out, splits=s, **kw_post)  # noqa
        cfg, splits = tuned_config(key, M, self.cout, run, K, dma, aligned, halo=halo,
                                   cgemm_only=self.post is not None, stem=self.c4)
        run(cfg, splits)
        return outs


class FusedDualConv:
    """``act(conv1x1(h) + conv1x1_stride(x) + b)`` as ONE GEMM over the
    K-concatenated operands [h | x(strided)] and weights [W_h ; W_x] (cgemm
    dual-source A mode): a ResNet bottleneck's expand conv and its projection
    shortcut, without writing / re-reading the projection's output."""

    def __init__(self, conv_h: FusedConv, conv_x: FusedConv, act: str, device, use_hip: bool, name: str):
        self.c1, self.c2 = conv_h.cin, conv_x.cin
        self.cout = conv_h.cout
        self.sh, self.sw = conv_x.sh, conv_x.sw
        self.act = act
        self.use_hip = use_hip
        self.name = name
        self.device = device
        if use_hip:
            # [Cout][C1 + C2] bf16, concatenated on the device (no host round trip)
            w = torch.cat([conv_h.w[:, :self.c1], conv_x.w[:, :self.c2]], dim=1)
            self.w = to_device(_pad_k(w, 8), device)
            self.b = (conv_h.b + conv_x.b).contiguous()
        else:
            self.w1, self.w2 = conv_h.w_ref, conv_x.w_ref
            self.b_ref = conv_h.b_ref + conv_x.b_ref

    post = None
    post_mode = None
    set_post = FusedConv.set_post

    def post_ok(self) -> bool:
        return self.cout % 8 == 0

    def __call__(self, ctx, node, ins):
        h, x = O.to_torch(ins[0]), O.to_torch(ins[1])
        if not self.use_hip:
            y = h.float() @ self.w1.reshape(self.c1, self.cout)
            xs = x.float()[:, ::self.sh, ::self.sw, :]
            y = y + xs @ self.w2.reshape(self.c2, self.cout) + self.b_ref
            return _with_post(self, _ref_act(y, self.act).contiguous())
        from ..ops import ACT, hip, tuned_config
        H = hip()
        h, x = _to_bf16(h).contiguous(), _to_bf16(x).contiguous()
        n, ho, wo, _ = h.shape
        out = torch.empty((n, ho, wo, self.cout), device=h.device, dtype=BF16)
        key = ("dual", tuple(h.shape), tuple(x.shape), self.cout, self.sh, self.act, self.post_mode)
        kw_post, outs = _post_kwargs(self, out)
        run = lambda c, s: H.conv2d_dual(h, x, self.w, self.b, self.sh, self.sw, ACT[self.act], c, out, s,  # noqa
                                         **kw_post)
        cfg, splits = tuned_config(key, n * ho * wo, self.cout, run, self.c1 + self.c2, True, True, cgemm_only=True)
        run(cfg, splits)
        return outs


class FusedMatMul:
    """``pad_n``: the consumers accept a row-strided [M, N] view, so an N that
    is not a multiple of 8 (ResNet's 1001 classes) is computed as ceil8(N)
    columns (zero weight rows) into an [M, ceil8(N)] buffer and returned as
    its first N columns: the pipelined cgemm kernel applies (it needs N % 8 ==
    0) instead of igemm + split-K reduce."""

    def __init__(self, w_kn: torch.Tensor, bias: Optional[torch.Tensor], act: str, out_f32: bool,
                 device, use_hip: bool, name: str, pad_n: bool = False):
        self.k, self.n = w_kn.shape
        self.act = act
        self.out_f32 = out_f32
        self.use_hip = use_hip and self.k % 8 == 0
        self.name = name
        b = bias if bias is not None else zeros(self.n, w_kn)
        self.np = -(-self.n // 8) * 8 if (pad_n and self.n % 8 and self.k % 64 == 0) else self.n
        self.device = device
        # the fp32 weights as given, kept until the compile passes are over
        # (defer_layernorm folds a LayerNorm's gamma / beta into them; then
        # release_weight_sources drops them)
        self._w_src = w_kn if self.use_hip else None
        if self.use_hip:
            w_nk = w_kn.t().contiguous()
            if self.np != self.n:
                w_nk = torch.cat([w_nk, torch.zeros(self.np - self.n, self.k, dtype=w_nk.dtype, device=w_nk.device)])
                b = torch.cat([b.float().reshape(-1), zeros(self.np - self.n, b)])
            self.w = to_device(_pad_k(w_nk, 8).to(BF16), device)
            self.b = to_device(b.float(), device)
        else:
            self.w_ref = to_device(w_kn.float(), device)
            self.b_ref = to_device(b.float(), device)

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        res = O.to_torch(ins[1]) if len(ins) > 1 else None
        if not self.use_hip:
            y = x.float() @ self.w_ref.to(x.device) + self.b_ref.to(x.device)
            if res is not None:
                y = y + res.float()
            y = _ref_act(y, self.act)
            return [y if self.out_f32 or not x.is_cuda else y.to(BF16)]
        from ..ops import ACT, hip, tuned_config
        H = hip()
        x = _to_bf16(x)
        if not (x.dim() == 2 and x.stride(1) == 1 and x.stride(0) % 8 == 0 and res is None):
            # (a row-strided 2-D view -- BERT's pooler reading each sequence's
            # first token out of [B, S, H] -- is read in place: no copy kernel)
            x = x.contiguous()
        if res is not None:
            res = _to_bf16(res).contiguous()
        M = x.shape[0] if x.dim() == 2 else x.numel() // self.k
        padded = self.np != self.n and res is None and x.dim() == 2
        n = self.np if padded else self.n
        w, b = (self.w, self.b) if padded or self.np == self.n else (self.w[:self.n], self.b[:self.n])
        shape = list(x.shape[:-1]) + [n]
        out = torch.empty(shape, device=x.device, dtype=torch.float32 if self.out_f32 else BF16)
        key = ("mm", M, n, self.k, res is not None, self.out_f32, self.act) + \
            ((x.stride(0),) if not x.is_contiguous() else ())
        run = lambda c, s: H.linear(x, w, b, res, ACT[self.act], c, self.out_f32, 1.0, out, s)  # noqa
        cfg, splits = tuned_config(key, M, n, run, self.k, True, self.k % 64 == 0)
        y = run(cfg, splits)
        return [y[:, :self.n] if padded else y]


class DeferredLNMatMul(FusedMatMul):
    """A _FusedMatMul / _FusedQKV around LayerNorms that are never stored
    (``defer_layernorm``): ``LN(z) = (z - mean) * rstd * gamma + beta`` of a
    GEMM output ``z`` is applied inside the GEMMs that read it, from row
    statistics the producing GEMM's epilogue emits ([M][P][2] fp32 (sum, sum of
    squares) partials, one per row and producer column block).

    * ``emit``: this GEMM's bf16 output rows feed a deferred LayerNorm: it also
      returns their partials (output 1).
    * ``a_ln`` = (eps,): input 0 is a pre-LayerNorm ``z`` (statistics at input
      ``a_pos``).  ``LN(z) @ W + b = rstd * (z @ W' - mean * colsum(W')) + b'``
      with ``W' = diag(gamma) W`` (folded in fp32, then rounded once to bf16),
      ``b' = b + beta @ W`` and ``colsum`` = the per-column sums of the bf16
      ``W'`` -- the GEMM runs on ``z`` unchanged.
    * ``r_ln`` = (gamma, beta, eps): the residual (input 1) is a pre-LayerNorm
      ``z`` (statistics at input ``r_pos``), normalised per element in the
      epilogue.

    One kernel per GEMM (kernels/cgemm_impl.h epilogue_lnx, bindings
    ``linear_lnx``): the 23 of 24 encoder LayerNorm launches of BERT-base
    whose inputs and outputs are GEMMs disappear (the last one feeds the
    pooler's strided view and stays).  Round 3's fold spilled registers in
    the 8-wave tiles (profiles/round3/ln_fold.md); this one does not (LDS
    column vectors, statistics fetched before the K loop, a separate LNX
    kernel build), and still only breaks even -- see defer_layernorm."""

    emit = False
    has_res = False
    a_ln = None
    a_pos = None
    r_ln = None
    r_pos = None
    colsum = None

    @classmethod
    def of(cls, node) -> "DeferredLNMatMul":
        """The node's impl as a DeferredLNMatMul (converted in place the first
        time, while its inputs are still [x] or [x, residual])."""
        mm = node.attr("_impl")
        if isinstance(mm, DeferredLNMatMul):
            return mm
        d = cls.__new__(cls)
        d.__dict__.update(mm.__dict__)
        d.has_res = len(node.inputs) > 1
        node.attrs["_impl"] = d
        return d

    def fold_input_ln(self, gamma: torch.Tensor, beta: torch.Tensor, eps: float):
        w_kn = self._w_src.float()
        g = gamma.detach().float().reshape(-1).to(w_kn.device)
        bt = beta.detach().float().reshape(-1).to(w_kn.device)
        b = self.b.detach().float().to(w_kn.device)
        wf = w_kn * g[:, None]
        self.w = to_device(_pad_k(wf.t().contiguous(), 8).to(BF16), self.device)
        self.b = to_device((b + bt @ w_kn).float(), self.device)
        self.colsum = self.w.float().sum(1).contiguous()
        self.a_ln = (float(eps),)

    def _stats(self, st: torch.Tensor, length: int, eps: float):
        s = st.float().sum(1)
        mean = s[:, 0] / length
        var = (s[:, 1] / length - mean * mean).clamp_min(0)
        return mean, torch.rsqrt(var + eps)

    def __call__(self, ctx, node, ins):
        x = _to_bf16(O.to_torch(ins[0])).contiguous()
        res = _to_bf16(O.to_torch(ins[1])).contiguous() if self.has_res else None
        a_st = O.to_torch(ins[self.a_pos]) if self.a_ln is not None else None
        r_st = O.to_torch(ins[self.r_pos]) if self.r_ln is not None else None
        M = x.numel() // self.k
        shape = list(x.shape[:-1]) + [self.n]
        if not x.is_cuda:
            return self._reference(x, res, a_st, r_st, M, shape)
        from ..ops import ACT, hip, tuned_config
        H = hip()
        out = torch.empty(shape, device=x.device, dtype=torch.float32 if self.out_f32 else BF16)
        ra = self.r_ln
        key = ("mmx", M, self.n, self.k, res is not None, self.out_f32, self.act, self.a_ln is not None,
               ra is not None, self.emit)

        def run(c, _s):
            return H.linear_lnx(x, self.w, self.b, res, ACT[self.act], c, self.out_f32, out,
                                a_st, self.colsum, self.a_ln[0] if self.a_ln else 1e-12,
                                r_st, ra[0] if ra else None, ra[1] if ra else None, ra[2] if ra else 1e-12,
                                self.emit)
        cfg, _ = tuned_config(key, M, self.n, run, self.k, True, True, no_split=True, ln=True)
        y, st = run(cfg, 1)
        return [y, st] if self.emit else [y]

    def _reference(self, x, res, a_st, r_st, M, shape):
        """The kernel's math in fp32 torch (CPU tensors; tests)."""
        acc = x.float().reshape(M, self.k) @ self.w.float().cpu()[:, :self.k].t()
        if self.a_ln is not None:
            mean, rstd = self._stats(a_st.cpu(), self.k, self.a_ln[0])
            acc = rstd[:, None] * (acc - mean[:, None] * self.colsum.cpu()[None, :])
        y = acc + self.b.float().cpu()
        if res is not None:
            r = res.float().reshape(M, self.n)
            if self.r_ln is not None:
                g, b, eps = self.r_ln
                mean, rstd = self._stats(r_st.cpu(), self.n, eps)
                r = (r - mean[:, None]) * rstd[:, None] * g.cpu() + b.cpu()
            y = y + r
        y = _ref_act(y, self.act)
        yb = y.to(BF16) if not self.out_f32 else y
        outs = [yb.reshape(shape)]
        if self.emit:
            f = yb.float()
            outs.append(torch.stack([f.sum(1), (f * f).sum(1)], 1).reshape(M, 1, 2))
        return outs


def _lnx_gemm_ok(impl, k: int) -> bool:
    return isinstance(impl, FusedMatMul) and impl.use_hip and impl.np == impl.n and impl.k == k and \
        impl.k % 64 == 0 and impl.n % 32 == 0 and getattr(impl, "_w_src", None) is not None


def defer_layernorm(g, order, fed, fetch_refs, device, opts):
    """_LayerNorm(z) with z = a _FusedMatMul output read by nothing else, and
    every reader of the LayerNorm a _FusedMatMul / _FusedQKV taking it as
    input 0 (A) or input 1 (residual): the LayerNorm node goes away -- the
    producer emits z's row statistics, the readers take z plus the
    statistics (DeferredLNMatMul).  Opt-in (TFSERVE_DEFER_LN=1): on
    MI355X it measured level with the LayerNorm kernels at b32 (engine
    1.560 / 1.568 vs 1.544 ms), behind at b1 (0.624 vs 0.585 ms) and in the
    BERT serving bench (25.9k vs 27.1k RPC/s, profiles/round5/s15): the
    epilogue work it adds to the four GEMMs (1.5-2.5 us each in isolation,
    scripts/lnx_probe.py) costs about what the LayerNorm launches did."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    if not c.use_hip or os.environ.get("TFSERVE_DEFER_LN", "0") != "1":
        return
    for name in order:
        ln_node = g.nodes.get(name)
        if ln_node is None or ln_node.op != "_LayerNorm" or ln_node.name in c.fetch_nodes:
            continue
        ln = ln_node.attr("_impl")
        if ln is None or not getattr(ln, "use_hip", False):
            continue
        C = ln.g.numel()
        src, sidx = ln_node.inputs[0]
        prod = g.nodes.get(src)
        if prod is None or sidx != 0 or prod.op not in ("_FusedMatMul", "_FusedQKV"):
            continue
        pm = prod.attr("_impl")
        if not isinstance(pm, FusedMatMul) or not pm.use_hip or pm.n != C or pm.np != C or pm.out_f32 or \
                pm.k % 64 or C % 32 or c.only_consumer(prod.name) is not ln_node:
            continue
        readers = c.cons.get(ln_node.name, [])
        ok = bool(readers)
        for cname, pos, oidx in readers:
            cn = g.nodes[cname]
            ci = cn.attr("_impl")
            if oidx != 0 or cn.op not in ("_FusedMatMul", "_FusedQKV") or ci is None:
                ok = False
            elif pos == 0:
                ok = ok and _lnx_gemm_ok(ci, C) and getattr(ci, "a_ln", None) is None and \
                    not (len(cn.inputs) > 1 and cn.inputs[1] == (ln_node.name, 0))
            elif pos == 1:
                ok = ok and isinstance(ci, FusedMatMul) and ci.use_hip and ci.n == C and ci.np == C and \
                    ci.k % 64 == 0 and ci.n % 32 == 0 and getattr(ci, "r_ln", None) is None
            else:
                ok = False
        if not ok:
            continue
        DeferredLNMatMul.of(prod).emit = True
        z = (prod.name, 0)
        stats = (prod.name, 1)
        for cname, pos, _o in readers:
            cn = g.nodes[cname]
            d = DeferredLNMatMul.of(cn)
            cn.inputs[pos] = z
            if pos == 0:
                d.fold_input_ln(ln.g, ln.b, ln.eps)
                d.a_pos = len(cn.inputs)
            else:
                d.r_ln = (ln.g, ln.b, float(ln.eps))
                d.r_pos = len(cn.inputs)
            cn.inputs.append(stats)
        del g.nodes[ln_node.name]
        c.refresh()


def ln_weight_frags(w_nk: torch.Tensor) -> torch.Tensor:
    """[N][K] -> the fragment-major layout kernels/lngemm.hip streams: for
    16-row n-tile nt and 32-deep K-step t, one contiguous KB whose lane l =
    16 q + r holds w[16 nt + r][32 t + 8 q .. + 8] (a v_mfma_f32_16x16x32_bf16
    B fragment).  Returned as a contiguous [N][K] tensor."""
    n, k = w_nk.shape
    return w_nk.reshape(n // 16, 16, k // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous().reshape(n, k)


class MatMulLN:
    """A _FusedMatMul with a residual input whose only reader is a _LayerNorm
    over its N columns (BERT's attention-output projection + residual +
    LayerNorm): one ``hip().linear_ln`` launch (kernels/lngemm.hip: a
    workgroup owns whole rows, so the row statistics stay on the CU and the
    GEMM output is never re-read), or the two launches -- timed per shape
    (ops.tuned_choice: option 0 = split, 1 / 2 / 3 = the fused kernel with
    32 / 64 / 16 rows per workgroup).  The weights stay in the children
    (parallel/weights.py binds them there).  Request path: BERT Predict
    (/root/reference/protos/tensorflow_serving/apis/predict.proto:12-40)."""

    children = ("mm", "ln")
    BM = {1: 32, 2: 64, 3: 16}

    def __init__(self, mm: "FusedMatMul", ln):
        self.mm, self.ln = mm, ln
        self.use_hip = mm.use_hip and ln.use_hip
        self.name = mm.name
        # the kernel's fragment-major copy of the weights (a weight of this op:
        # built from mm.w on its device, meta on a follower until bound)
        self.w_frag = ln_weight_frags(mm.w[:, :mm.k])

    @staticmethod
    def fusable(mm, ln) -> bool:
        from ..ops import hip
        return isinstance(mm, FusedMatMul) and mm.use_hip and getattr(ln, "use_hip", False) and \
            mm.act == "none" and not mm.out_f32 and mm.np == mm.n and mm.n == ln.g.numel() and \
            mm.n in (512, 768, 1024) and mm.k % 128 == 0 and hip().linear_ln_supported(1, mm.n, mm.k, 32)

    def __call__(self, ctx, node, ins):
        mm, ln = self.mm, self.ln

        def split():
            return ln(ctx, node, mm(ctx, node, ins))
        x = O.to_torch(ins[0])
        res = O.to_torch(ins[1]) if len(ins) > 1 else None
        if not (self.use_hip and x.is_cuda and x.shape[-1] == mm.k and (res is None or res.shape[-1] == mm.n)):
            return split()
        from ..ops import hip, tuned_choice
        H = hip()
        xb = _to_bf16(x).contiguous()
        rb = None if res is None else _to_bf16(res).contiguous()
        M = xb.numel() // mm.k
        opts = {0: split}
        for o, bm in self.BM.items():
            if H.linear_ln_supported(M, mm.n, mm.k, bm):
                opts[o] = (lambda bm=bm: [H.linear_ln(xb, self.w_frag, mm.b, rb, ln.g, ln.b, ln.eps, bm)])
        key = ("mmln", M, mm.n, mm.k, rb is not None)
        pick = tuned_choice(key, opts, default=0)
        return opts.get(pick, split)()


def fuse_matmul_layernorm(g, order, fed, fetch_refs, device, opts):
    """_LayerNorm(_FusedMatMul(x, residual)) with the LayerNorm the GEMM
    output's only reader -> _FusedMatMulLN (MatMulLN).  GPU only, opt-in
    (TFSERVE_MATMUL_LN=1): measured slower than the two launches on MI355X.
    BERT-base b32 attention output (4096 x 768 x 768, graph-captured, L2-cold
    operands): fused 21.1 us (16 rows per workgroup) / 23.2 us (32) against
    11.9 + 5.8 = 17.7 us; FFN2 (K = 3072) 63.2 against 37.5 us
    (profiles/round6/r6j/probe.log).  A workgroup that owns whole rows must
    stream the whole weight matrix (1.2 MB) through one CU, and one CU takes in
    ~60 GB/s even with fragment-major weights (42-46 us per workgroup with
    [N][K] fragment loads, profiles/round6/r6h).  The opt-in defer_layernorm
    (TFSERVE_DEFER_LN=1) takes precedence."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    if not c.use_hip or os.environ.get("TFSERVE_MATMUL_LN", "0") != "1" or \
            os.environ.get("TFSERVE_DEFER_LN", "0") == "1":
        return
    for name in order:
        ln_node = g.nodes.get(name)
        if ln_node is None or ln_node.op != "_LayerNorm" or len(ln_node.inputs) != 1:
            continue
        src, sidx = ln_node.inputs[0]
        prod = g.nodes.get(src)
        if prod is None or sidx != 0 or prod.op != "_FusedMatMul" or c.only_consumer(prod.name) is not ln_node:
            continue
        mm, ln = prod.attr("_impl"), ln_node.attr("_impl")
        if ln is None or not MatMulLN.fusable(mm, ln):
            continue
        ln_node.op = "_FusedMatMulLN"
        ln_node.attrs = {"_impl": MatMulLN(mm, ln)}
        ln_node.inputs = list(prod.inputs)
        ln_node.ctrl = _merge_ctrl([prod, ln_node])
        del g.nodes[prod.name]
        c.refresh()


def release_weight_sources(g, order, fed, fetch_refs, device, opts):
    """Drops the fp32 weight copies the GEMM ops kept for defer_layernorm."""
    for n in g.nodes.values():
        impl = n.attrs.get("_impl") if n.attrs else None
        if isinstance(impl, FusedMatMul):
            impl._w_src = None


class DenseSoftmax:
    """softmax(x @ W + b) over a few classes (BERT's classifier: 2 labels):
    one kernel (misc.hip dense_softmax_kernel) from the fp32 pooled rows,
    instead of cast + a GEMM launch with mostly empty tiles + torch softmax."""
    children = ("mm",)          # placement.weight_refs: the classifier weights live in mm

    def __init__(self, mm: "FusedMatMul"):
        self.mm = mm

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        mm = self.mm
        if mm.use_hip and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.is_contiguous() and \
                mm.k % 4 == 0:
            from ..ops import hip
            return [hip().dense_softmax(x, mm.w, mm.b, mm.n)]
        y = mm(ctx, node, [x])[0]
        return [torch.softmax(y.float(), dim=-1)]


def fuse_dense_softmax(g, order, fed, fetch_refs, device, opts):
    """Softmax(_FusedMatMul(x)) with <= 16 classes, no activation / residual and
    the logits used by nothing else -> _DenseSoftmax(x)."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        sm = g.nodes.get(name)
        if sm is None or sm.op != "Softmax" or len(sm.inputs) != 1:
            continue
        mm = g.nodes.get(sm.inputs[0][0])
        if mm is None or mm.op != "_FusedMatMul" or sm.inputs[0][1] != 0 or len(mm.inputs) != 1:
            continue
        impl = mm.attrs.get("_impl")
        if impl is None or impl.n > 16 or impl.act != "none" or c.only_consumer(mm.name) is not sm:
            continue
        sm.op = "_DenseSoftmax"
        sm.inputs = [mm.inputs[0]]
        sm.ctrl = _merge_ctrl([mm, sm])
        sm.attrs = {"_impl": DenseSoftmax(impl)}
        del g.nodes[mm.name]
        c.refresh()


def _with_post(impl, y: torch.Tensor) -> list:
    """CPU reference of the post-activation output: [y] / [y, post] / [post]."""
    if impl.post is None:
        return [y]
    scale, shift, act = impl.post
    z = _ref_act(y * scale.to(y.device) + shift.to(y.device), act).contiguous()
    return [y, z] if impl.post_mode == "dual" else [z]


def _post_kwargs(impl, out: torch.Tensor):
    """(kernel kwargs, op outputs) for the fused post-activation output."""
    if impl.post is None:
        return {}, [out]
    from ..ops import ACT
    scale, shift, act = impl.post
    if impl.post_mode == "dual":
        out2 = torch.empty_like(out)
        return dict(post_scale=scale, post_shift=shift, post_act=ACT[act], out2=out2), [out, out2]
    return dict(post_scale=scale, post_shift=shift, post_act=ACT[act], post_only=True), [out]


def _ref_act(y, act):
    if act == "relu":
        return torch.relu(y)
    if act == "tanh":
        return torch.tanh(y)
    if act == "gelu_tanh":
        return F.gelu(y, approximate="tanh")
    if act == "gelu_erf":
        return F.gelu(y)
    return y


def _impl_op(ctx, node, ins):
    return node.attrs["_impl"](ctx, node, ins)


for _op in ("_FusedConv2D", "_FusedDualConv", "_FusedMatMul", "_GlobalAvgPool", "_MaxPool",
            "_SoftmaxArgMax", "_LayerNorm",
            "_FusedQKV", "_Attention", "_EmbeddingLN", "_KeyMaskAdder", "_DenseSoftmax"):
    O.OPS[_op] = _impl_op


class GlobalAvgPool:
    def __init__(self, keep_dims: bool, use_hip: bool):
        self.keep = keep_dims
        self.use_hip = use_hip

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if self.use_hip and x.is_cuda and x.shape[-1] % 8 == 0:
            from ..ops import hip
            y = hip().global_avgpool(_to_bf16(x).contiguous())
        else:
            y = x.float().mean(dim=(1, 2))
        return [y.reshape(y.shape[0], 1, 1, -1) if self.keep else y]


class MaxPool:
    def __init__(self, ksize, strides, padding, use_hip):
        self.kh, self.kw = ksize
        self.sh, self.sw = strides
        self.padding = padding
        self.use_hip = use_hip
        self.post = None
        self.post_mode = None

    def set_post(self, scale, shift, act, mode, device=None):
        # on the device up front: a host->device copy inside HIP-graph capture is illegal
        dev = device if (self.use_hip and device is not None) else "cpu"
        self.post = (to_device(scale.float(), dev), to_device(shift.float(), dev), act)
        self.post_mode = mode

    def post_ok(self) -> bool:
        return True

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        h, w = x.shape[1], x.shape[2]
        if self.padding == "SAME":
            (pt, pb), (pl, pr) = O.tf_same_pads(h, self.kh, self.sh), O.tf_same_pads(w, self.kw, self.sw)
        else:
            pt = pb = pl = pr = 0
        if self.use_hip and x.is_cuda and x.shape[-1] % 8 == 0 and self.post_mode != "dual":
            from ..ops import ACT, hip
            kw = {}
            if self.post is not None:    # folded BN (+ReLU) after the max, same kernel
                sc, sh, act = self.post
                kw = dict(post_scale=sc, post_shift=sh, post_act=ACT[act])
            return [hip().maxpool(_to_bf16(x).contiguous(), self.kh, self.kw, self.sh, self.sw, pt, pb, pl, pr,
                                  **kw)]
        xc = F.pad(x.permute(0, 3, 1, 2), [pl, pr, pt, pb], value=float("-inf"))
        y = F.max_pool2d(xc, (self.kh, self.kw), (self.sh, self.sw)).permute(0, 2, 3, 1).contiguous()
        return _with_post(self, y)


class SoftmaxArgMax:
    def __init__(self, use_hip, classes_dtype):
        self.use_hip = use_hip
        self.cdt = classes_dtype

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if self.use_hip and x.is_cuda and x.dim() == 2 and x.dtype in (torch.float32, BF16):
            from ..ops import hip
            if x.stride(-1) != 1:
                x = x.contiguous()
            probs, cls = hip().softmax_argmax(x, True, True)     # row-strided views are fine
        else:
            probs = torch.softmax(x.float(), dim=-1)
            cls = torch.argmax(x.float(), dim=-1)
        return [probs, cls if self.cdt == torch.int64 else cls.to(self.cdt)]


class ClassifierHead:
    """``_GlobalAvgPool -> _FusedMatMul (no act) -> _SoftmaxArgMax`` (the ResNet
    head) as two launches (``hip().classifier_head``: pooled split-K partial
    dot products, then bias + partial sums + softmax/argmax) instead of three
    with a 16-workgroup, 2048-deep serial GEMM in the middle."""

    def __init__(self, mm: FusedMatMul, classes_dtype, use_hip: bool):
        self.n = mm.n
        self.cdt = classes_dtype
        self.use_hip = use_hip and mm.use_hip and mm.k in (512, 1024, 2048, 4096)
        if mm.use_hip:
            self.w, self.b = mm.w, mm.b                     # bf16 [Np][K], f32 [Np]
        else:
            self.w_ref, self.b_ref = mm.w_ref, mm.b_ref     # f32 [K][N], [N]

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        if self.use_hip and x.is_cuda and x.dim() == 4 and x.shape[-1] == self.w.shape[1]:
            from ..ops import current_head_host_rows, hip
            rows = current_head_host_rows()
            if rows is not None:
                # a serving lane's capture: the one-launch head also writes
                # the lane's pinned output rows (ops.head_host_rows)
                p_ptr = rows[0] if rows[1] == self.n else 0
                c_ptr = rows[2] if self.cdt == torch.int64 else 0
                probs, cls, wrote = hip().classifier_head_to_host(_to_bf16(x).contiguous(), self.w, self.b, self.n,
                                                                  p_ptr, c_ptr)
                if wrote:
                    probs._tfs_host, cls._tfs_host = p_ptr, c_ptr
                return [probs, cls]
            probs, cls = hip().classifier_head(_to_bf16(x).contiguous(), self.w, self.b, self.n)
        else:
            pooled = x.float().mean(dim=(1, 2))
            if hasattr(self, "w_ref"):
                logits = pooled @ self.w_ref.to(x.device) + self.b_ref.to(x.device)
            else:
                logits = (pooled @ self.w.float().t().to(x.device) + self.b.to(x.device))[:, :self.n]
            probs = torch.softmax(logits, dim=-1)
            cls = torch.argmax(logits, dim=-1)
        return [probs, cls if self.cdt == torch.int64 else cls.to(self.cdt)]


O.OPS["_ClassifierHead"] = _impl_op


class StemPool:
    """``_FusedConv2D(7x7/2, RGB) -> _MaxPool(3x3/2)`` (the ResNet stem) as ONE
    kernel (``hip().stem_pool``, kernels/stem.hip): the fp32 request is read
    directly, the conv output stays in LDS and only the pooled map is written
    (three launches and two passes over the 112x112x64 conv output before)."""

    children = ("conv", "pool")        # weight_refs (graph/placement.py) walks these

    def __init__(self, conv: FusedConv, pool: MaxPool):
        self.conv, self.pool = conv, pool
        self.use_hip = conv.use_hip and conv.c4

    def accepts_bf16_input(self, pos: int) -> bool:
        """The kernel rounds the request to bf16 before its MFMAs: a request
        already rounded the same way on ingest gives identical results."""
        return pos == 0 and self.use_hip

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        conv, pool = self.conv, self.pool
        if not (self.use_hip and x.is_cuda and x.dim() == 4):
            return pool(ctx, node, conv(ctx, node, [x]))
        from ..ops import ACT, hip
        pt, pb, pl, pr = conv.pads_for(x.shape[1], x.shape[2])
        hc = (x.shape[1] + pt + pb - conv.kh) // conv.sh + 1
        wc = (x.shape[2] + pl + pr - conv.kw) // conv.sw + 1
        if pool.padding == "SAME":
            (ppt, ppb), (ppl, ppr) = O.tf_same_pads(hc, 3, 2), O.tf_same_pads(wc, 3, 2)
        else:
            ppt = ppb = ppl = ppr = 0
        kw = {}
        if pool.post is not None:
            sc, sh, act = pool.post
            kw = dict(post_scale=sc, post_shift=sh, post_act=ACT[act])
        x = x.contiguous() if x.dtype == torch.bfloat16 else x.float().contiguous()
        return [hip().stem_pool(x, conv.w, conv.b, pt, pb, pl, pr, ACT[conv.act],
                                ppt, ppb, ppl, ppr, **kw)]


O.OPS["_StemPool"] = _impl_op

# (K1, N1, N2) shapes kernels/chain.hip is built for (ResNet-50 stages 1-2).
# Stage 2's (N1 = 512) pairs measured no faster chained than as two launches
# at b32 (each workgroup re-reads 256-384 KB of weights for 64 rows, one
# workgroup per CU: profiles/round3/conv_chain.md); since round 5 every shape
# is chained in the graph and ChainConv times the chain against the two
# convs per batch bucket (ops.tuned_choice), so each bucket runs its faster
# form.  TFSERVE_CONV_CHAIN_SHAPES=stage1 restores the stage-1-only pass.
CHAIN_SHAPES_ALL = {(64, 256, 64), (64, 256, 128), (128, 512, 128), (128, 512, 256)}
CHAIN_SHAPES_STAGE1 = {(64, 256, 64), (64, 256, 128)}
CHAIN_SHAPES_DEFAULT = CHAIN_SHAPES_ALL


class ChainConv:
    """A bottleneck's expand 1x1 conv (+ shortcut, act) and the NEXT
    bottleneck's reduce 1x1 conv (+ act), which reads exactly its output, as
    one kernel (``hip().conv_chain``, kernels/chain.hip): outputs
    ``[y1, y2]``; y1 (the block output, also the next shortcut) is written
    once and never read back by the reduce.  SURVEY.md S8 fused conv epilogues;
    the request path is the reference client's ResNet Predict
    (/root/reference/src/lib.rs:229-257)."""

    children = ("a", "b")

    def __init__(self, a: FusedConv, b: FusedConv):
        self.a, self.b = a, b
        self.use_hip = a.use_hip and b.use_hip
        self.name = a.name

    def __call__(self, ctx, node, ins):
        x = O.to_torch(ins[0])
        res = O.to_torch(ins[1]) if len(ins) > 1 else None
        a, b = self.a, self.b

        def split():
            y1 = a(ctx, node, ins)[0]
            return [y1, b(ctx, node, [y1])[0]]
        if not (self.use_hip and x.is_cuda and x.dim() == 4 and x.shape[-1] == a.cin):
            return split()
        from ..ops import ACT, hip, tuned_choice
        xb = _to_bf16(x).contiguous()
        rb = None if res is None else _to_bf16(res).contiguous()

        def chained():
            return list(hip().conv_chain(xb, a.w, a.b, rb, ACT[a.act], b.w, b.b, ACT[b.act]))
        # one workgroup per 64 rows: the chain wins where it saves a launch
        # boundary at small row counts or re-reads of large Y1 tiles, and loses
        # where 64-row workgroups leave CUs idle -- timed per shape (bucket):
        # option 1 = the chain kernel, 0 = the two convs with their own tiles
        key = ("chain", tuple(x.shape), a.cout, b.cout, res is not None, a.act, b.act)
        # without a tuned pick (TFSERVE_AUTOTUNE=0, no committed table, or a
        # key the table lacks) only the stage-1 shapes chain: the stage-2
        # (N1 = 512) chains measured no faster than two convs at b32
        # (round-5 ADVICE)
        dflt = 1 if (a.cin, a.cout, b.cout) in CHAIN_SHAPES_STAGE1 else 0
        pick = tuned_choice(key, {1: chained, 0: split}, default=dflt)
        return chained() if pick == 1 else split()


O.OPS["_ChainConv"] = _impl_op
O.OPS["_FusedMatMulLN"] = _impl_op

_PASSTHROUGH = ("Identity", "Squeeze", "Reshape")


# ------------------------------------------------------------------ passes
def fuse_classifier_head(g, order, fed, fetch_refs, device, opts):
    """_SoftmaxArgMax(dense(mean_hw(x))) -> _ClassifierHead(x); every node in
    between must have that single consumer and not be fetched."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)

    def single(node) -> bool:
        return node.name not in c.fetch_nodes and len(c.cons.get(node.name, [])) == 1

    def walk(ref, chain):
        n = g.nodes.get(ref[0])
        while n is not None and n.op in _PASSTHROUGH and ref[1] == 0 and single(n) and n.inputs:
            chain.append(n)
            ref = n.inputs[0]
            n = g.nodes.get(ref[0])
        return ref, n

    for name in order:
        sm = g.nodes.get(name)
        if sm is None or sm.op != "_SoftmaxArgMax" or not sm.inputs:
            continue
        chain: List[Node] = []
        ref, mm = walk(sm.inputs[0], chain)
        if mm is None or mm.op != "_FusedMatMul" or ref[1] != 0 or len(mm.inputs) != 1 or not single(mm):
            continue
        impl = mm.attrs["_impl"]
        if impl.act != "none":
            continue
        chain.append(mm)
        ref, gap = walk(mm.inputs[0], chain)
        if gap is None or gap.op != "_GlobalAvgPool" or ref[1] != 0 or not single(gap):
            continue
        chain.append(gap)
        sm_impl = sm.attrs["_impl"]
        head = ClassifierHead(impl, sm_impl.cdt, c.use_hip)
        sm.op = "_ClassifierHead"
        sm.inputs = [gap.inputs[0]]
        sm.attrs = {"_impl": head}
        sm.ctrl = _merge_ctrl(chain + [sm])
        for n in chain:
            del g.nodes[n.name]
        c.refresh()


def fuse_stem_pool(g, order, fed, fetch_refs, device, opts):
    """``_MaxPool(3x3/2)(_FusedConv2D(7x7/2, C <= 4 channels, 16..64 outputs))``
    -> ``_StemPool`` when the conv has no residual / post output and feeds only
    the pool, and the pool writes a single output."""
    import os
    if os.environ.get("TFSERVE_STEM_POOL", "1") == "0":       # A/B switch
        return
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        p = g.nodes.get(name)
        if p is None or p.op != "_MaxPool" or not p.inputs or p.inputs[0][1] != 0:
            continue
        pool = p.attrs["_impl"]
        if (pool.kh, pool.kw, pool.sh, pool.sw) != (3, 3, 2, 2) or pool.post_mode == "dual":
            continue
        cn = g.nodes.get(p.inputs[0][0])
        if cn is None or cn.op != "_FusedConv2D" or len(cn.inputs) != 1 or c.only_consumer(cn.name) is not p:
            continue
        conv = cn.attrs["_impl"]
        if not isinstance(conv, FusedConv) or (conv.kh, conv.kw, conv.sh, conv.sw) != (7, 7, 2, 2) or \
                conv.cin > 4 or conv.cout % 16 or not 16 <= conv.cout <= 64 or conv.post is not None or \
                conv.act not in ("none", "relu"):
            continue
        if c.use_hip and not conv.c4:
            continue
        p.op = "_StemPool"
        p.inputs = [cn.inputs[0]]
        p.ctrl = _merge_ctrl([cn, p])
        p.attrs = {"_impl": StemPool(conv, pool)}
        del g.nodes[cn.name]
        c.refresh()


def fuse_conv(g, order, fed, fetch_refs, device, opts):
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        n = g.nodes.get(name)
        if n is None or n.op != "Conv2D" or n.sattr("data_format", "NHWC") != "NHWC":
            continue
        dil = n.attr("dilations", [1, 1, 1, 1]) or [1, 1, 1, 1]
        if any(d != 1 for d in dil):
            continue
        w = _const(g, n.inputs[1])
        if w is None or w.dim() != 4:
            continue
        x_ref = n.inputs[0]
        padding = n.sattr("padding", "VALID")
        pads = (0, 0, 0, 0)
        chain: List[Node] = []
        if padding == "EXPLICIT":
            ep = n.attr("explicit_paddings", [])
            if ep[0] or ep[1] or ep[6] or ep[7]:
                continue
            pads = (ep[2], ep[3], ep[4], ep[5])
        prod = g.nodes.get(x_ref[0])
        if (padding == "VALID" and prod is not None and prod.op == "Pad" and x_ref[1] == 0
                and c.only_consumer(prod.name) is n):
            pv = _const(g, prod.inputs[1])
            if pv is not None:
                p = [int(v) for v in pv.reshape(-1).tolist()]
                if p[0] == p[1] == p[6] == p[7] == 0 and min(p) >= 0:
                    chain.append(prod)
                    x_ref = prod.inputs[0]
                    padding, pads = "EXPLICIT", (p[2], p[3], p[4], p[5])
        strides = n.attr("strides", [1, 1, 1, 1])
        w = w.float()
        cout = w.shape[3]
        bias = zeros(cout, w)
        chain.append(n)
        cur = n
        residual = None
        act = "none"
        nxt = c.only_consumer(cur.name)
        if nxt is not None and nxt.op == "BiasAdd" and nxt.inputs[0] == (cur.name, 0):
            b = _const(g, nxt.inputs[1])
            if b is not None and b.numel() == cout:
                bias = bias + b.float()
                chain.append(nxt)
                cur = nxt
                nxt = c.only_consumer(cur.name)
        if (nxt is not None and nxt.op in ("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3")
                and not nxt.attr("is_training", False) and nxt.sattr("data_format", "NHWC") == "NHWC"
                and nxt.inputs[0] == (cur.name, 0)):
            params = [_const(g, r) for r in nxt.inputs[1:5]]
            outs_used = {i for _c, _p, i in c.cons.get(nxt.name, [])}
            if all(p is not None for p in params) and outs_used <= {0} and nxt.name not in c.fetch_nodes:
                gamma, beta, mean, var = (p.float() for p in params)
                scale = gamma * torch.rsqrt(var + float(nxt.attr("epsilon", 1e-3)))
                w = w * scale
                bias = (bias - mean) * scale + beta
                chain.append(nxt)
                cur = nxt
                nxt = c.only_consumer(cur.name)
        # a constant per-channel / scalar scale (ResNet v2's residual scale):
        # folded into the weights and bias
        if nxt is not None and nxt.op == "Mul" and len(nxt.inputs) == 2 and (cur.name, 0) in nxt.inputs:
            other = nxt.inputs[1] if nxt.inputs[0] == (cur.name, 0) else nxt.inputs[0]
            sv = _const(g, other)
            if sv is not None and sv.numel() in (1, cout) and other != (cur.name, 0):
                sv = sv.float().reshape(-1)
                w = w * sv
                bias = bias * sv
                chain.append(nxt)
                cur = nxt
                nxt = c.only_consumer(cur.name)
        if nxt is not None and nxt.op in ("Add", "AddV2") and len(nxt.inputs) == 2:
            other = nxt.inputs[1] if nxt.inputs[0] == (cur.name, 0) else nxt.inputs[0]
            if other != (cur.name, 0) and _const(g, other) is None:
                residual = other
                chain.append(nxt)
                cur = nxt
                nxt = c.only_consumer(cur.name)
        if nxt is not None and nxt.op == "Relu":
            act = "relu"
            chain.append(nxt)
            cur = nxt
        impl = FusedConv(w, bias, (strides[1], strides[2]), padding, pads, act, device, c.use_hip, cur.name)
        inputs = [x_ref] + ([residual] if residual is not None else [])
        _finalize(g, chain, "_FusedConv2D", inputs, {"_impl": impl})
        c.refresh()


def _feeds_head(c: _Ctx, name: str, depth: int = 0) -> bool:
    if name in c.fetch_nodes:
        return True
    if depth > 3:
        return False
    for cname, _p, _i in c.cons.get(name, []):
        cn = c.g.nodes[cname]
        if cn.op in ("Softmax", "ArgMax", "_SoftmaxArgMax", "LogSoftmax", "TopKV2", "Sigmoid"):
            return True
        if cn.op in ("Identity", "Squeeze", "Reshape") and _feeds_head(c, cname, depth + 1):
            return True
    return False


GELU_ACTS = ("gelu_tanh", "gelu_erf")


def fuse_matmul(g, order, fed, fetch_refs, device, opts):
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        n = g.nodes.get(name)
        if n is None or n.op != "MatMul" or n.attr("transpose_a", False):
            continue
        w = _const(g, n.inputs[1])
        if w is None or w.dim() != 2:
            continue
        w = w.float()
        if n.attr("transpose_b", False):
            w = w.t()
        kdim, ndim = w.shape
        chain = [n]
        cur = n
        bias = None
        residual = None
        act = "none"
        nxt = c.only_consumer(cur.name)
        if nxt is not None and nxt.op in ("BiasAdd", "Add", "AddV2") and nxt.inputs[0] == (cur.name, 0):
            b = _const(g, nxt.inputs[1])
            if b is not None and b.numel() == ndim:
                bias = b.float().reshape(-1)
                chain.append(nxt)
                cur = nxt
                nxt = c.only_consumer(cur.name)
        gelu = match_gelu(g, c, cur.name)
        if gelu is not None:
            act, gnodes, out_node = gelu
            chain += gnodes + [out_node]
            cur = out_node
        elif nxt is not None and nxt.op in ("Relu", "Tanh"):
            act = nxt.op.lower()
            chain.append(nxt)
            cur = nxt
        elif nxt is not None and nxt.op in ("Add", "AddV2") and len(nxt.inputs) == 2:
            other = nxt.inputs[1] if nxt.inputs[0] == (cur.name, 0) else nxt.inputs[0]
            if other != (cur.name, 0) and _const(g, other) is None:
                residual = other
                chain.append(nxt)
                cur = nxt
        out_f32 = _feeds_head(c, cur.name)
        cons = c.cons.get(cur.name, [])
        pad_n = cur.name not in c.fetch_nodes and bool(cons) and \
            all(g.nodes[cn].op == "_SoftmaxArgMax" for cn, _p, _i in cons)
        impl = FusedMatMul(w, bias, act, out_f32, device, c.use_hip, cur.name, pad_n)
        _finalize(g, chain, "_FusedMatMul", [n.inputs[0]] + ([residual] if residual else []), {"_impl": impl})
        c.refresh()


def match_gelu(g: Graph, c: _Ctx, src: str):
    """Match GELU applied to ``src`` (exactly-once uses):
    erf form:  0.5 * x * (1 + erf(x / sqrt(2)))   (any association order)
    tanh form: 0.5 * x * (1 + tanh(sqrt(2/pi) * (x + 0.044715 * x^3)))
    Returns (act, interior nodes, output node) or None."""
    from .patterns import match_gelu_subgraph
    return match_gelu_subgraph(g, c, src)


def fuse_pools(g, order, fed, fetch_refs, device, opts):
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        n = g.nodes.get(name)
        if n is None:
            continue
        if n.op == "Mean":
            ax = _const(g, n.inputs[1])
            if ax is not None and sorted(int(a) for a in ax.reshape(-1).tolist()) in ([1, 2], [-3, -2]):
                n.op = "_GlobalAvgPool"
                n.attrs = {"_impl": GlobalAvgPool(bool(n.attr("keep_dims", False)), c.use_hip)}
                n.inputs = [n.inputs[0]]
        elif n.op == "MaxPool" and n.sattr("data_format", "NHWC") == "NHWC":
            k, s = n.attr("ksize"), n.attr("strides")
            n.op = "_MaxPool"
            n.attrs = {"_impl": MaxPool((k[1], k[2]), (s[1], s[2]), n.sattr("padding", "VALID"), c.use_hip)}


def fuse_softmax_argmax(g, order, fed, fetch_refs, device, opts):
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    by_input: Dict[tuple, Dict[str, Node]] = {}
    for name in order:
        n = g.nodes.get(name)
        if n is None or not n.inputs:
            continue
        if n.op == "Softmax":
            by_input.setdefault(n.inputs[0], {})["sm"] = n
        elif n.op == "ArgMax":
            ax = _const(g, n.inputs[1])
            if ax is not None and ax.numel() == 1 and int(ax.reshape(-1)[0]) in (1, -1):
                by_input.setdefault(n.inputs[0], {})["am"] = n
    for src, d in by_input.items():
        if "sm" in d and "am" in d:
            sm, am = d["sm"], d["am"]
            cdt = O.DT_TO_TORCH.get(am.attrs.get("output_type", T.DT_INT64), torch.int64)
            sm.op = "_SoftmaxArgMax"
            sm.attrs = {"_impl": SoftmaxArgMax(c.use_hip, cdt)}
            am.op = "Identity"
            am.inputs = [(sm.name, 1)]
            am.attrs = {}


def _is_1x1(impl) -> bool:
    """A 1x1 conv without padding (SAME never pads a 1x1 filter)."""
    return isinstance(impl, FusedConv) and impl.kh == impl.kw == 1 and impl.use_hip and not impl.c4 and \
        (impl.padding != "EXPLICIT" or not any(impl.pads))


def fuse_dual_conv(g, order, fed, fetch_refs, device, opts):
    """Merge ``_FusedConv2D(a, residual=_FusedConv2D(b))`` where both are 1x1
    convs, the residual producer has no activation and no other consumer, and
    one of them has stride 1, into ``_FusedDualConv(h=stride-1 input, x=other
    input)`` (GPU only; both channel counts multiples of 64)."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    if not c.use_hip:
        return
    for name in order:
        n = g.nodes.get(name)
        if n is None or n.op != "_FusedConv2D" or len(n.inputs) != 2:
            continue
        a = n.attrs["_impl"]
        r = g.nodes.get(n.inputs[1][0])
        if r is None or r.op != "_FusedConv2D" or len(r.inputs) != 1 or n.inputs[1][1] != 0:
            continue
        b = r.attrs["_impl"]
        if not (_is_1x1(a) and _is_1x1(b)) or b.act != "none" or c.only_consumer(r.name) is not n:
            continue
        if a.cin % 64 or b.cin % 64 or a.cout != b.cout or a.cout % 8:
            continue
        # the stride-1 conv's input is the dense source (its rows are the output pixels)
        if a.sh == a.sw == 1:
            conv_h, h_ref, conv_x, x_ref = a, n.inputs[0], b, r.inputs[0]
        elif b.sh == b.sw == 1:
            conv_h, h_ref, conv_x, x_ref = b, r.inputs[0], a, n.inputs[0]
        else:
            continue
        impl = FusedDualConv(conv_h, conv_x, a.act, device, c.use_hip, n.name)
        n.op = "_FusedDualConv"
        n.inputs = [h_ref, x_ref]
        n.ctrl = _merge_ctrl([r, n])
        n.attrs = {"_impl": impl}
        del g.nodes[r.name]
        c.refresh()


def _bn_affine(g: Graph, c: _Ctx, bn: Node):
    """(scale, shift) of an inference FusedBatchNorm with constant params whose
    only used output is y, else None."""
    if bn.op not in ("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3") or bn.attr("is_training", False) \
            or bn.sattr("data_format", "NHWC") != "NHWC" or bn.name in c.fetch_nodes:
        return None
    params = [_const(g, r) for r in bn.inputs[1:5]]
    if any(p is None for p in params) or {i for _c, _p, i in c.cons.get(bn.name, [])} - {0}:
        return None
    gamma, beta, mean, var = (p.float().reshape(-1) for p in params)
    scale = gamma * torch.rsqrt(var + float(bn.attr("epsilon", 1e-3)))
    return scale, beta - mean * scale


def fuse_post_activation(g, order, fed, fetch_refs, device, opts):
    """ResNet v2 pre-activation: ``P -> FusedBatchNorm -> [Relu]`` where P is a
    fused conv / dual conv / max-pool becomes a second output of P written by
    the same kernel's epilogue: P then yields ``[sum, relu(bn(sum))]`` when the
    raw sum has other consumers (the next block's identity shortcut), or just
    ``[relu(bn(sum))]`` when it does not (a projecting next block; the final
    post-norm before the global pool).  SURVEY.md §2.7 K1's dual-output
    epilogue; the model is the reference's ``resnet_v2_fp32_savedmodel_NHWC``
    (``serving/fetch.sh:7``)."""
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    for name in order:
        p = g.nodes.get(name)
        if p is None or p.op not in ("_FusedConv2D", "_FusedDualConv", "_MaxPool"):
            continue
        impl = p.attrs["_impl"]
        if impl.post is not None or not impl.post_ok() or name in c.fetch_nodes:
            continue
        cons = c.cons.get(name, [])
        if any(i != 0 for _c, _p, i in cons):
            continue
        bns = [g.nodes[cn] for cn, _pos, _i in cons
               if g.nodes[cn].op.startswith("FusedBatchNorm") and g.nodes[cn].inputs[0] == (name, 0)]
        if len(bns) != 1:
            continue
        bn = bns[0]
        aff = _bn_affine(g, c, bn)
        if aff is None or aff[0].numel() != getattr(impl, "cout", aff[0].numel()):
            continue
        out_node, act = bn, "none"
        relu = c.only_consumer(bn.name)
        if relu is not None and relu.op == "Relu" and relu.name not in c.fetch_nodes:
            out_node, act = relu, "relu"
        elif bn.name in c.fetch_nodes:
            continue
        others = [cn for cn, _pos, _i in cons if cn != bn.name]
        if isinstance(impl, MaxPool) and others:
            continue                  # the pooling kernel writes one output
        mode = "dual" if others else "only"
        if isinstance(impl, MaxPool):
            impl.set_post(aff[0], aff[1], act, mode, device=c.device)
        else:
            impl.set_post(aff[0], aff[1], act, mode)
        new_ref = (name, 1 if mode == "dual" else 0)
        for cn, pos, _i in c.cons.get(out_node.name, []):
            g.nodes[cn].inputs[pos] = new_ref
        p.ctrl = _merge_ctrl([p, bn] + ([out_node] if out_node is not bn else []))
        del g.nodes[bn.name]
        if out_node is not bn:
            del g.nodes[out_node.name]
        c.refresh()


def _chainable_1x1(impl) -> bool:
    return (isinstance(impl, FusedConv) and impl.kh == 1 and impl.kw == 1 and impl.sh == 1 and impl.sw == 1 and
            not impl.c4 and impl.post is None and impl.act in ("relu", "none") and
            (impl.padding != "EXPLICIT" or not any(impl.pads)))


def fuse_conv_chain(g, order, fed, fetch_refs, device, opts):
    """``_FusedConv2D`` A (1x1 expand, optional residual) whose output feeds a
    ``_FusedConv2D`` B (1x1 reduce, no residual) -> ``_ChainConv`` with outputs
    ``[A, B]`` when (A.cin, A.cout, B.cout) is a kernel shape; A's other
    consumers (the next shortcut) keep reading output 0.  GPU programs only
    (``TFSERVE_CONV_CHAIN=0`` disables it, ``force`` applies it on CPU too:
    the op then runs both reference convs)."""
    import os
    mode = os.environ.get("TFSERVE_CONV_CHAIN", "1")
    shapes = CHAIN_SHAPES_STAGE1 if os.environ.get("TFSERVE_CONV_CHAIN_SHAPES") == "stage1" else CHAIN_SHAPES_ALL
    c = _Ctx(g, order, fed, fetch_refs, device, opts)
    if mode == "0" or (not c.use_hip and mode != "force"):
        return
    for name in order:
        p = g.nodes.get(name)
        if p is None or p.op != "_FusedConv2D" or name in c.fetch_nodes:
            continue
        a = p.attrs["_impl"]
        if not _chainable_1x1(a):
            continue
        cons = c.cons.get(name, [])
        if any(i != 0 for _c, _p, i in cons):
            continue
        bs = [g.nodes[cn] for cn, pos, _i in cons
              if pos == 0 and g.nodes[cn].op == "_FusedConv2D" and len(g.nodes[cn].inputs) == 1 and
              cn not in c.fetch_nodes and _chainable_1x1(g.nodes[cn].attrs["_impl"])]
        if len(bs) != 1:
            continue
        bnode = bs[0]
        b = bnode.attrs["_impl"]
        if b.cin != a.cout or (a.cin, a.cout, b.cout) not in shapes:
            continue
        chain = ChainConv(a, b)
        p.op = "_ChainConv"
        p.attrs = {"_impl": chain}
        for cn, pos, _i in c.cons.get(bnode.name, []):
            g.nodes[cn].inputs[pos] = (name, 1)
        p.ctrl = _merge_ctrl([p, bnode])
        del g.nodes[bnode.name]
        c.refresh()


def default_passes(options=None):
    from .patterns import bert_passes, late_passes
    return [fuse_pools, fuse_softmax_argmax] + bert_passes() + [fuse_conv, fuse_dual_conv, fuse_post_activation,
                                                                 fuse_stem_pool, fuse_matmul,
                                                                 fuse_classifier_head, fuse_dense_softmax,
                                                                 fuse_conv_chain] + late_passes() + \
        [fuse_matmul_layernorm, defer_layernorm, release_weight_sources]
