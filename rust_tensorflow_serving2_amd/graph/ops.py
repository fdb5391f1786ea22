"""Reference op library: TF op semantics on torch tensors.

Every op the loader meets is executed here unless a fusion pass replaced it
with a fused HIP op (``graph/fused.py``).  These kernels define correctness:
fused/HIP paths are tested against them.  Conventions:

* numeric tensors are ``torch.Tensor`` on the executor's device (fp32 math for
  float ops); DT_STRING tensors are numpy object arrays (host only);
* small integer tensors that only feed shapes (``Shape``, shape constants,
  reduction axes ...) stay on the CPU so a graph can be captured into a HIP
  graph without host syncs — ``host_ints`` reads them.
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from ..utils import tensors as T
from .ir import Node

DT_TO_TORCH = {
    T.DT_FLOAT: torch.float32, T.DT_DOUBLE: torch.float64, T.DT_INT32: torch.int32,
    T.DT_UINT8: torch.uint8, T.DT_INT16: torch.int16, T.DT_INT8: torch.int8,
    T.DT_INT64: torch.int64, T.DT_BOOL: torch.bool, T.DT_HALF: torch.float16,
    T.DT_BFLOAT16: torch.bfloat16, T.DT_COMPLEX64: torch.complex64,
    T.DT_COMPLEX128: torch.complex128,
}
TORCH_TO_DT = {v: k for k, v in DT_TO_TORCH.items()}


class OpError(ValueError):
    """Bad inputs for an op at run time (INVALID_ARGUMENT)."""


class Unsupported(NotImplementedError):
    pass


OPS: Dict[str, Callable] = {}
# ops whose outputs stay on the host (shape arithmetic)
HOST_OPS = {"Shape", "ShapeN", "Size", "Rank"}


def op(*names):
    def deco(fn):
        for n in names:
            OPS[n] = fn
        return fn
    return deco


class Ctx:
    """Per-run execution context."""

    def __init__(self, device: torch.device):
        self.device = device

    def tensor(self, x, dtype=None):
        if isinstance(x, torch.Tensor):
            return x
        return torch.as_tensor(np.asarray(x), dtype=dtype)


def to_torch(v, device=None) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        return v if device is None or v.device == device else v.to(device)
    a = np.asarray(v)
    if a.dtype == np.uint16:
        t = torch.from_numpy(a.astype(np.int32)).to(torch.int32)
    else:
        t = torch.from_numpy(np.require(a, requirements="C"))
    return t if device is None else t.to(device)


def host_ints(v) -> List[int]:
    if isinstance(v, torch.Tensor):
        return [int(x) for x in v.detach().reshape(-1).cpu().tolist()]
    return [int(x) for x in np.asarray(v).reshape(-1).tolist()]


def host_int(v) -> int:
    xs = host_ints(v)
    if len(xs) != 1:
        raise OpError(f"expected a scalar, got {len(xs)} values")
    return xs[0]


def dt_attr(node: Node, key: str, default=T.DT_FLOAT) -> torch.dtype:
    dt = node.attrs.get(key, default)
    if dt is None:
        dt = default
    if dt not in DT_TO_TORCH:
        raise Unsupported(f"{node.op}: dtype {T.DT_NAMES.get(dt, dt)} not supported")
    return DT_TO_TORCH[dt]


def _same_device(a: torch.Tensor, b: torch.Tensor):
    if a.device != b.device:
        if a.device.type == "cpu":
            a = a.to(b.device)
        else:
            b = b.to(a.device)
    return a, b


# ------------------------------------------------------------------ leaves
@op("Const")
def _const(ctx, n, ins):
    return [n.value[0]]


@op("Identity", "StopGradient", "Snapshot", "PreventGradient", "CheckNumerics",
    "EnsureShape", "ReadVariableOp", "PlaceholderWithDefault", "DebugIdentity")
def _identity(ctx, n, ins):
    return [ins[0]]


@op("IdentityN")
def _identity_n(ctx, n, ins):
    return list(ins)


@op("NoOp")
def _noop(ctx, n, ins):
    return []


@op("Placeholder")
def _placeholder(ctx, n, ins):
    raise OpError(f"You must feed a value for placeholder tensor '{n.name}'")


# ------------------------------------------------------------------ elementwise
def _binary(fn):
    def impl(ctx, n, ins):
        if any(isinstance(x, np.ndarray) and x.dtype == object for x in ins):
            raise Unsupported(f"{n.op} on strings")
        a, b = to_torch(ins[0]), to_torch(ins[1])
        a, b = _same_device(a, b)
        return [fn(a, b)]
    return impl


for _name, _fn in {
    "Add": torch.add, "AddV2": torch.add, "Sub": torch.sub, "Mul": torch.mul,
    "Maximum": torch.maximum, "Minimum": torch.minimum, "Pow": torch.pow,
    "SquaredDifference": lambda a, b: (a - b) * (a - b),
    "Equal": torch.eq, "NotEqual": torch.ne, "Less": torch.lt, "LessEqual": torch.le,
    "Greater": torch.gt, "GreaterEqual": torch.ge, "LogicalAnd": torch.logical_and,
    "LogicalOr": torch.logical_or, "BiasAddV1": torch.add,
}.items():
    OPS[_name] = _binary(_fn)


@op("RealDiv", "Div")
def _div(ctx, n, ins):
    a, b = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    if not a.is_floating_point() and n.op == "Div":
        return [torch.div(a, b, rounding_mode="trunc")]
    return [a / b]


@op("FloorDiv")
def _floordiv(ctx, n, ins):
    a, b = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    return [torch.div(a, b, rounding_mode="floor")]


@op("FloorMod")
def _floormod(ctx, n, ins):
    a, b = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    return [torch.remainder(a, b)]


def _unary(fn):
    def impl(ctx, n, ins):
        return [fn(to_torch(ins[0]))]
    return impl


for _name, _fn in {
    "Relu": torch.relu, "Relu6": lambda x: torch.clamp(x, 0, 6), "Tanh": torch.tanh,
    "Sigmoid": torch.sigmoid, "Exp": torch.exp, "Log": torch.log, "Sqrt": torch.sqrt,
    "Rsqrt": torch.rsqrt, "Square": lambda x: x * x, "Neg": torch.neg, "Abs": torch.abs,
    "Erf": torch.erf, "Floor": torch.floor, "Ceil": torch.ceil, "Round": torch.round,
    "Reciprocal": torch.reciprocal, "Inv": torch.reciprocal, "Sign": torch.sign,
    "Softplus": F.softplus, "Softsign": F.softsign, "Elu": F.elu, "Selu": F.selu,
    "LogicalNot": torch.logical_not, "Log1p": torch.log1p, "Expm1": torch.expm1,
    "Sin": torch.sin, "Cos": torch.cos, "IsNan": torch.isnan, "Gelu": F.gelu,
}.items():
    OPS[_name] = _unary(_fn)


@op("LeakyRelu")
def _leaky(ctx, n, ins):
    return [F.leaky_relu(to_torch(ins[0]), float(n.attr("alpha", 0.2)))]


@op("AddN")
def _addn(ctx, n, ins):
    out = to_torch(ins[0])
    for x in ins[1:]:
        out = out + to_torch(x).to(out.device)
    return [out]


@op("BiasAdd")
def _bias_add(ctx, n, ins):
    x, b = to_torch(ins[0]), to_torch(ins[1])
    if n.sattr("data_format", "NHWC") == "NCHW" and x.dim() > 2:
        shape = [1, -1] + [1] * (x.dim() - 2)
        return [x + b.reshape(shape)]
    return [x + b]


@op("Cast")
def _cast(ctx, n, ins):
    dt = dt_attr(n, "DstT")
    x = ins[0]
    if isinstance(x, np.ndarray) and x.dtype == object:
        raise Unsupported("Cast of strings")
    return [to_torch(x).to(dt)]


@op("Select", "SelectV2")
def _select(ctx, n, ins):
    c, a, b = to_torch(ins[0]), to_torch(ins[1]), to_torch(ins[2])
    dev = a.device if a.device.type != "cpu" else b.device
    c, a, b = c.to(dev), a.to(dev), b.to(dev)
    if n.op == "Select" and c.dim() == 1 and a.dim() > 1:
        c = c.reshape([-1] + [1] * (a.dim() - 1))
    return [torch.where(c, a, b)]


# ------------------------------------------------------------------ shapes
@op("Shape")
def _shape(ctx, n, ins):
    dt = dt_attr(n, "out_type", T.DT_INT32)
    return [torch.tensor(list(_shape_of(ins[0])), dtype=dt)]


@op("ShapeN")
def _shape_n(ctx, n, ins):
    dt = dt_attr(n, "out_type", T.DT_INT32)
    return [torch.tensor(list(_shape_of(x)), dtype=dt) for x in ins]


def _shape_of(x):
    return tuple(x.shape)


@op("Size")
def _size(ctx, n, ins):
    dt = dt_attr(n, "out_type", T.DT_INT32)
    return [torch.tensor(int(np.prod(_shape_of(ins[0]))), dtype=dt)]


@op("Rank")
def _rank(ctx, n, ins):
    return [torch.tensor(len(_shape_of(ins[0])), dtype=torch.int32)]


def _resolve_reshape(shape: List[int], numel: int) -> List[int]:
    if -1 in shape:
        known = 1
        for d in shape:
            if d != -1:
                known *= d
        shape = [numel // known if d == -1 and known else d for d in shape]
    return shape


@op("Reshape")
def _reshape(ctx, n, ins):
    x = ins[0]
    shape = host_ints(ins[1])
    if isinstance(x, np.ndarray):
        return [x.reshape(shape)]
    x = to_torch(x)
    try:
        return [x.reshape(shape)]
    except RuntimeError as e:
        raise OpError(f"{n.name}: cannot reshape {list(x.shape)} to {shape}: {e}") from None


@op("Squeeze")
def _squeeze(ctx, n, ins):
    x = ins[0]
    dims = n.attr("squeeze_dims", []) or []
    shape = list(x.shape)
    if dims:
        nd = len(shape)
        dims = sorted({d % nd for d in dims})
        new = [s for i, s in enumerate(shape) if i not in dims]
    else:
        new = [s for s in shape if s != 1]
    return [x.reshape(new)]


@op("ExpandDims")
def _expand(ctx, n, ins):
    x = ins[0]
    ax = host_int(ins[1])
    if isinstance(x, np.ndarray):
        return [np.expand_dims(x, ax)]
    return [to_torch(x).unsqueeze(ax if ax >= 0 else ax + to_torch(x).dim() + 1)]


@op("Transpose")
def _transpose(ctx, n, ins):
    perm = host_ints(ins[1])
    x = ins[0]
    if isinstance(x, np.ndarray):
        return [np.transpose(x, perm)]
    return [to_torch(x).permute(perm).contiguous()]


@op("ConcatV2")
def _concat(ctx, n, ins):
    ax = host_int(ins[-1])
    xs = ins[:-1]
    if all(isinstance(x, np.ndarray) and x.dtype == object for x in xs):
        return [np.concatenate(xs, axis=ax)]
    ts = [to_torch(x) for x in xs]
    dev = next((t.device for t in ts if t.device.type != "cpu"), ts[0].device)
    return [torch.cat([t.to(dev) for t in ts], dim=ax)]


@op("Concat")
def _concat_v1(ctx, n, ins):
    ax = host_int(ins[0])
    ts = [to_torch(x) for x in ins[1:]]
    dev = next((t.device for t in ts if t.device.type != "cpu"), ts[0].device)
    return [torch.cat([t.to(dev) for t in ts], dim=ax)]


@op("Pack")
def _pack(ctx, n, ins):
    ax = int(n.attr("axis", 0))
    ts = [to_torch(x) for x in ins]
    dev = next((t.device for t in ts if t.device.type != "cpu"), ts[0].device)
    return [torch.stack([t.to(dev) for t in ts], dim=ax)]


@op("Unpack")
def _unpack(ctx, n, ins):
    ax = int(n.attr("axis", 0))
    return list(torch.unbind(to_torch(ins[0]), dim=ax))


@op("Fill")
def _fill(ctx, n, ins):
    shape = host_ints(ins[0])
    v = to_torch(ins[1])
    return [torch.full(shape, v.item() if v.device.type == "cpu" else 0, dtype=v.dtype,
                       device=v.device) if v.device.type == "cpu" else v.expand(shape).clone()]


@op("ZerosLike")
def _zeros_like(ctx, n, ins):
    return [torch.zeros_like(to_torch(ins[0]))]


@op("OnesLike")
def _ones_like(ctx, n, ins):
    return [torch.ones_like(to_torch(ins[0]))]


@op("Range")
def _range(ctx, n, ins):
    s, l, d = (to_torch(x).item() for x in ins)
    dt = dt_attr(n, "Tidx", T.DT_INT32)
    return [torch.arange(s, l, d, dtype=dt)]


@op("Tile")
def _tile(ctx, n, ins):
    return [to_torch(ins[0]).repeat(host_ints(ins[1]))]


@op("Slice")
def _slice(ctx, n, ins):
    x = to_torch(ins[0])
    begin, size = host_ints(ins[1]), host_ints(ins[2])
    idx = tuple(slice(b, x.shape[i] if s == -1 else b + s) for i, (b, s) in enumerate(zip(begin, size)))
    return [x[idx]]


@op("StridedSlice")
def _strided_slice(ctx, n, ins):
    x = ins[0]
    begin, end, strides = host_ints(ins[1]), host_ints(ins[2]), host_ints(ins[3])
    bm, em = int(n.attr("begin_mask", 0)), int(n.attr("end_mask", 0))
    elm, nam, sam = int(n.attr("ellipsis_mask", 0)), int(n.attr("new_axis_mask", 0)), int(n.attr("shrink_axis_mask", 0))
    idx = []
    for i in range(len(begin)):
        bit = 1 << i
        if elm & bit:
            idx.append(Ellipsis)
        elif nam & bit:
            idx.append(None)
        elif sam & bit:
            idx.append(begin[i])
        else:
            b = None if bm & bit else begin[i]
            e = None if em & bit else end[i]
            idx.append(slice(b, e, strides[i]))
    if isinstance(x, np.ndarray):
        return [x[tuple(idx)]]
    t = to_torch(x)
    if any(isinstance(s, slice) and s.step is not None and s.step < 0 for s in idx):
        # torch has no negative steps: go through numpy on host for small tensors
        return [torch.from_numpy(np.require(t.cpu().numpy()[tuple(idx)], requirements="C")).to(t.device)]
    return [t[tuple(idx)]]


@op("Split")
def _split(ctx, n, ins):
    ax = host_int(ins[0])
    k = int(n.attr("num_split"))
    return list(torch.chunk(to_torch(ins[1]), k, dim=ax))


@op("SplitV")
def _splitv(ctx, n, ins):
    sizes = host_ints(ins[1])
    ax = host_int(ins[2])
    x = to_torch(ins[0])
    if -1 in sizes:
        i = sizes.index(-1)
        sizes[i] = x.shape[ax] - (sum(sizes) + 1)
    return list(torch.split(x, sizes, dim=ax))


@op("Pad", "PadV2", "MirrorPad")
def _pad(ctx, n, ins):
    x = to_torch(ins[0])
    pads = host_ints(ins[1])
    pairs = [(pads[2 * i], pads[2 * i + 1]) for i in range(len(pads) // 2)]
    flat = []
    for b, e in reversed(pairs):
        flat += [b, e]
    if n.op == "MirrorPad":
        mode = n.sattr("mode", "REFLECT").lower()
        return [F.pad(x.permute(0, 3, 1, 2), flat[:4], mode="reflect" if mode == "reflect" else "replicate")
                .permute(0, 2, 3, 1)]
    val = float(to_torch(ins[2]).item()) if n.op == "PadV2" else 0.0
    return [F.pad(x, flat, value=val)]


@op("GatherV2", "Gather")
def _gather(ctx, n, ins):
    params, idx = to_torch(ins[0]), to_torch(ins[1])
    ax = host_int(ins[2]) if n.op == "GatherV2" else 0
    batch_dims = int(n.attr("batch_dims", 0))
    if batch_dims:
        raise Unsupported("GatherV2 with batch_dims")
    if ax < 0:
        ax += params.dim()
    if idx.device.type == "cpu" and idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= params.shape[ax]):
        raise OpError(f"{n.name}: indices out of range [0, {params.shape[ax]})")
    idx = idx.to(params.device).long()
    if params.is_cuda:
        # no host sync (HIP-graph capturable): out-of-range rows read as zeros, as TF's GPU kernel does
        n_ax = params.shape[ax]
        valid = (idx >= 0) & (idx < n_ax)
        out = torch.index_select(params, ax, idx.clamp(0, n_ax - 1).reshape(-1))
        vshape = [1] * ax + [idx.numel()] + [1] * (params.dim() - ax - 1)
        out = out * valid.reshape(vshape).to(out.dtype)
    else:
        out = torch.index_select(params, ax, idx.reshape(-1))
    shape = list(params.shape[:ax]) + list(idx.shape) + list(params.shape[ax + 1:])
    return [out.reshape(shape)]


@op("ResourceGather")
def _rgather(ctx, n, ins):
    params, idx = to_torch(ins[0]), to_torch(ins[1]).to(to_torch(ins[0]).device).long()
    out = torch.index_select(params, 0, idx.reshape(-1))
    return [out.reshape(list(idx.shape) + list(params.shape[1:]))]


@op("OneHot")
def _onehot(ctx, n, ins):
    idx = to_torch(ins[0]).long()
    depth = host_int(ins[1])
    on, off = to_torch(ins[2]), to_torch(ins[3])
    ax = int(n.attr("axis", -1))
    valid = (idx >= 0) & (idx < depth)
    oh = F.one_hot(idx.clamp(0, depth - 1), depth) * valid.unsqueeze(-1)
    out = oh.to(on.dtype) * on.to(idx.device) + (1 - oh.to(on.dtype)) * off.to(idx.device)
    if ax != -1:
        out = out.movedim(-1, ax)
    return [out]


# ------------------------------------------------------------------ reductions
def _reduce(fn):
    def impl(ctx, n, ins):
        x = to_torch(ins[0])
        axes = host_ints(ins[1])
        keep = bool(n.attr("keep_dims", False))
        if not axes:
            return [x.clone()]
        axes = sorted({a % x.dim() for a in axes}) if x.dim() else []
        return [fn(x, axes, keep)]
    return impl


OPS["Mean"] = _reduce(lambda x, a, k: x.float().mean(dim=a, keepdim=k).to(x.dtype)
                      if not x.is_floating_point() else x.mean(dim=a, keepdim=k))
OPS["Sum"] = _reduce(lambda x, a, k: x.sum(dim=a, keepdim=k))
OPS["Prod"] = _reduce(lambda x, a, k: _prod(x, a, k))
OPS["Max"] = _reduce(lambda x, a, k: x.amax(dim=a, keepdim=k))
OPS["Min"] = _reduce(lambda x, a, k: x.amin(dim=a, keepdim=k))
OPS["All"] = _reduce(lambda x, a, k: x.bool().all(dim=a[0], keepdim=k) if len(a) == 1 else x.bool().all())
OPS["Any"] = _reduce(lambda x, a, k: x.bool().any(dim=a[0], keepdim=k) if len(a) == 1 else x.bool().any())


def _prod(x, axes, keep):
    for a in sorted(axes, reverse=True):
        x = x.prod(dim=a, keepdim=keep)
    return x


@op("ArgMax", "ArgMin")
def _argmax(ctx, n, ins):
    x = to_torch(ins[0])
    ax = host_int(ins[1])
    out = torch.argmax(x, dim=ax) if n.op == "ArgMax" else torch.argmin(x, dim=ax)
    return [out.to(dt_attr(n, "output_type", T.DT_INT64))]


@op("Softmax")
def _softmax(ctx, n, ins):
    x = to_torch(ins[0])
    return [torch.softmax(x.float(), dim=-1).to(x.dtype)]


@op("LogSoftmax")
def _log_softmax(ctx, n, ins):
    x = to_torch(ins[0])
    return [torch.log_softmax(x.float(), dim=-1).to(x.dtype)]


@op("TopKV2")
def _topk(ctx, n, ins):
    x = to_torch(ins[0])
    k = host_int(ins[1])
    v, i = torch.topk(x, k, dim=-1, largest=True, sorted=True)
    return [v, i.to(torch.int32)]


# ------------------------------------------------------------------ linear algebra
@op("MatMul")
def _matmul(ctx, n, ins):
    a, b = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    if n.attr("transpose_a", False):
        a = a.t()
    if n.attr("transpose_b", False):
        b = b.t()
    return [a @ b]


@op("BatchMatMul", "BatchMatMulV2", "BatchMatMulV3")
def _bmm(ctx, n, ins):
    a, b = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    if n.attr("adj_x", False):
        a = a.transpose(-1, -2)
    if n.attr("adj_y", False):
        b = b.transpose(-1, -2)
    return [torch.matmul(a, b)]


def tf_same_pads(in_size: int, k: int, s: int, d: int = 1):
    out = (in_size + s - 1) // s
    eff = (k - 1) * d + 1
    total = max((out - 1) * s + eff - in_size, 0)
    return total // 2, total - total // 2


def conv_pads(n: Node, h, w, kh, kw, sh, sw, dh=1, dw=1):
    pad = n.sattr("padding", "VALID")
    if pad == "SAME":
        return tf_same_pads(h, kh, sh, dh), tf_same_pads(w, kw, sw, dw)
    if pad == "EXPLICIT":
        ep = n.attr("explicit_paddings", [])
        # NHWC order: [N0,N1,H0,H1,W0,W1,C0,C1]
        return (ep[2], ep[3]), (ep[4], ep[5])
    return (0, 0), (0, 0)


def _nhwc(n: Node, x: torch.Tensor, fmt_key="data_format"):
    return n.sattr(fmt_key, "NHWC") != "NCHW"


@op("Conv2D")
def _conv2d(ctx, n, ins):
    x, w = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    nhwc = _nhwc(n, x)
    strides = n.attr("strides", [1, 1, 1, 1])
    dil = n.attr("dilations", [1, 1, 1, 1]) or [1, 1, 1, 1]
    if nhwc:
        sh, sw, dh, dw = strides[1], strides[2], dil[1], dil[2]
        xc = x.permute(0, 3, 1, 2)
    else:
        sh, sw, dh, dw = strides[2], strides[3], dil[2], dil[3]
        xc = x
    kh, kw, cin, cout = w.shape
    (pt, pb), (pl, pr) = conv_pads(n, xc.shape[2], xc.shape[3], kh, kw, sh, sw, dh, dw)
    groups = xc.shape[1] // cin
    xc = F.pad(xc, [pl, pr, pt, pb]) if (pt or pb or pl or pr) else xc
    y = F.conv2d(xc, w.permute(3, 2, 0, 1), stride=(sh, sw), dilation=(dh, dw), groups=groups)
    return [y.permute(0, 2, 3, 1).contiguous() if nhwc else y]


@op("DepthwiseConv2dNative")
def _dwconv(ctx, n, ins):
    x, w = _same_device(to_torch(ins[0]), to_torch(ins[1]))
    strides = n.attr("strides", [1, 1, 1, 1])
    nhwc = _nhwc(n, x)
    xc = x.permute(0, 3, 1, 2) if nhwc else x
    sh, sw = (strides[1], strides[2]) if nhwc else (strides[2], strides[3])
    kh, kw, cin, mult = w.shape
    (pt, pb), (pl, pr) = conv_pads(n, xc.shape[2], xc.shape[3], kh, kw, sh, sw)
    xc = F.pad(xc, [pl, pr, pt, pb])
    wt = w.permute(2, 3, 0, 1).reshape(cin * mult, 1, kh, kw)
    y = F.conv2d(xc, wt, stride=(sh, sw), groups=cin)
    return [y.permute(0, 2, 3, 1).contiguous() if nhwc else y]


def _pool_geom(n: Node, x):
    k = n.attr("ksize")
    s = n.attr("strides")
    nhwc = _nhwc(n, x)
    if nhwc:
        return nhwc, (k[1], k[2]), (s[1], s[2])
    return nhwc, (k[2], k[3]), (s[2], s[3])


@op("MaxPool")
def _maxpool(ctx, n, ins):
    x = to_torch(ins[0])
    nhwc, (kh, kw), (sh, sw) = _pool_geom(n, x)
    xc = x.permute(0, 3, 1, 2) if nhwc else x
    (pt, pb), (pl, pr) = conv_pads(n, xc.shape[2], xc.shape[3], kh, kw, sh, sw)
    if pt or pb or pl or pr:
        xc = F.pad(xc, [pl, pr, pt, pb], value=float("-inf"))
    y = F.max_pool2d(xc, (kh, kw), (sh, sw))
    return [y.permute(0, 2, 3, 1).contiguous() if nhwc else y]


@op("AvgPool")
def _avgpool(ctx, n, ins):
    x = to_torch(ins[0])
    nhwc, (kh, kw), (sh, sw) = _pool_geom(n, x)
    xc = x.permute(0, 3, 1, 2) if nhwc else x
    (pt, pb), (pl, pr) = conv_pads(n, xc.shape[2], xc.shape[3], kh, kw, sh, sw)
    xp = F.pad(xc, [pl, pr, pt, pb])
    ones = F.pad(torch.ones_like(xc[:, :1]), [pl, pr, pt, pb])
    s = F.avg_pool2d(xp, (kh, kw), (sh, sw)) * (kh * kw)
    c = F.avg_pool2d(ones, (kh, kw), (sh, sw)) * (kh * kw)
    y = s / c
    return [y.permute(0, 2, 3, 1).contiguous() if nhwc else y]


@op("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3")
def _fbn(ctx, n, ins):
    x = to_torch(ins[0])
    scale, offset, mean, var = (to_torch(t).to(x.device) for t in ins[1:5])
    eps = float(n.attr("epsilon", 1e-3))
    if n.attr("is_training", False):
        raise Unsupported(f"{n.name}: FusedBatchNorm with is_training=True cannot be served")
    nhwc = n.sattr("data_format", "NHWC") != "NCHW"
    inv = torch.rsqrt(var.float() + eps) * scale.float()
    shift = offset.float() - mean.float() * inv
    if not nhwc:
        inv = inv.reshape(1, -1, 1, 1)
        shift = shift.reshape(1, -1, 1, 1)
    y = (x.float() * inv + shift).to(x.dtype)
    outs = [y, mean, var, mean, var]
    if n.op == "FusedBatchNormV3":
        outs.append(torch.empty(0, device=x.device))
    return outs


# ------------------------------------------------------------------ tf.Example parsing
def _parse_examples(serialized, dense_keys, dense_defaults, dense_types, dense_shapes, node_name):
    from ..schema import tf as tfpb
    ser = np.asarray(serialized, dtype=object).reshape(-1)
    outs = []
    parsed = []
    for s in ser:
        try:
            parsed.append(tfpb.Example.FromString(bytes(s)))
        except Exception:
            raise OpError(f"{node_name}: could not parse example input") from None
    for key, dflt, dt, shp in zip(dense_keys, dense_defaults, dense_types, dense_shapes):
        k = key.decode() if isinstance(key, bytes) else key
        nelem = int(np.prod(shp)) if shp else 1
        rows = []
        for i, ex in enumerate(parsed):
            feat = ex.features.feature.get(k) if k in ex.features.feature else None
            if feat is None or feat.WhichOneof("kind") is None:
                d = np.asarray(dflt)
                if d.size == 0:
                    raise OpError(f"Name: <unknown>, Feature: {k} (data type: "
                                  f"{T.DT_NAMES.get(dt, dt)[3:].lower()}) is required but could not be found.")
                rows.append(np.broadcast_to(d.reshape(-1), (nelem,)) if d.size == 1 else d.reshape(-1))
                continue
            kind = feat.WhichOneof("kind")
            if dt == T.DT_FLOAT:
                if kind != "float_list":
                    raise OpError(f"Feature: {k}: data type mismatch (expected float)")
                vals = np.asarray(feat.float_list.value, np.float32)
            elif dt == T.DT_INT64:
                if kind != "int64_list":
                    raise OpError(f"Feature: {k}: data type mismatch (expected int64)")
                vals = np.asarray(feat.int64_list.value, np.int64)
            elif dt == T.DT_STRING:
                if kind != "bytes_list":
                    raise OpError(f"Feature: {k}: data type mismatch (expected bytes)")
                vals = np.empty(len(feat.bytes_list.value), dtype=object)
                vals[:] = list(feat.bytes_list.value)
            else:
                raise Unsupported(f"ParseExample dense type {dt}")
            if vals.size != nelem:
                raise OpError(f"Name: <unknown>, Key: {k}, Index: {i}.  Number of float values != "
                              f"expected.  values size: {vals.size} but output shape: {list(shp)}")
            rows.append(vals)
        arr = np.stack(rows).reshape([len(parsed)] + list(shp)) if rows else \
            np.zeros([0] + list(shp), dtype=T.np_dtype(dt))
        outs.append(arr if dt == T.DT_STRING else torch.from_numpy(np.require(arr, requirements="C")))
    return outs


@op("ParseExample")
def _parse_example(ctx, n, ins):
    nsparse, ndense = int(n.attr("Nsparse", 0)), int(n.attr("Ndense", 0))
    if nsparse:
        raise Unsupported("ParseExample with sparse features")
    dense_keys = [np.asarray(ins[2 + nsparse + i]).reshape(-1)[0] for i in range(ndense)]
    defaults = ins[2 + nsparse + ndense: 2 + nsparse + 2 * ndense]
    defaults = [d.cpu().numpy() if isinstance(d, torch.Tensor) else np.asarray(d) for d in defaults]
    outs = _parse_examples(ins[0], dense_keys, defaults, n.attr("Tdense", []), n.attr("dense_shapes", []), n.name)
    return outs


@op("ParseExampleV2")
def _parse_example_v2(ctx, n, ins):
    nsparse = int(n.attr("num_sparse", 0))
    if nsparse or n.attr("ragged_value_types"):
        raise Unsupported("ParseExampleV2 with sparse/ragged features")
    dense_keys = list(np.asarray(ins[3]).reshape(-1))
    tdense = n.attr("Tdense", [])
    defaults = ins[5:5 + len(tdense)]
    defaults = [d.cpu().numpy() if isinstance(d, torch.Tensor) else np.asarray(d) for d in defaults]
    return _parse_examples(ins[0], dense_keys, defaults, tdense, n.attr("dense_shapes", []), n.name)
