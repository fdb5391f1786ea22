"""TensorProto <-> numpy conversion (TF semantics), plus the zero-copy
PredictRequest decode that sits on top of the native codec.

TF rules honoured (tensor.proto, reference protos/tensorflow/core/framework/
tensor.proto:26-28): ``tensor_content`` wins when present; otherwise the typed
repeated field for the dtype is used, and if it holds fewer values than the
shape needs, the *last* value is repeated (a single value fills the tensor).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..schema import tf

DT_FLOAT, DT_DOUBLE, DT_INT32, DT_UINT8, DT_INT16, DT_INT8 = 1, 2, 3, 4, 5, 6
DT_STRING, DT_COMPLEX64, DT_INT64, DT_BOOL = 7, 8, 9, 10
DT_BFLOAT16, DT_UINT16, DT_COMPLEX128, DT_HALF, DT_UINT32, DT_UINT64 = 14, 17, 18, 19, 22, 23

# numpy has no bfloat16: carried as raw uint16 bits on the host.
DT_TO_NP = {
    DT_FLOAT: np.float32, DT_DOUBLE: np.float64, DT_INT32: np.int32, DT_UINT8: np.uint8,
    DT_INT16: np.int16, DT_INT8: np.int8, DT_COMPLEX64: np.complex64, DT_INT64: np.int64,
    DT_BOOL: np.bool_, DT_BFLOAT16: np.uint16, DT_UINT16: np.uint16,
    DT_COMPLEX128: np.complex128, DT_HALF: np.float16, DT_UINT32: np.uint32,
    DT_UINT64: np.uint64, DT_STRING: np.object_,
}
NP_TO_DT = {
    np.dtype(np.float32): DT_FLOAT, np.dtype(np.float64): DT_DOUBLE, np.dtype(np.int32): DT_INT32,
    np.dtype(np.uint8): DT_UINT8, np.dtype(np.int16): DT_INT16, np.dtype(np.int8): DT_INT8,
    np.dtype(np.complex64): DT_COMPLEX64, np.dtype(np.int64): DT_INT64, np.dtype(np.bool_): DT_BOOL,
    np.dtype(np.uint16): DT_UINT16, np.dtype(np.complex128): DT_COMPLEX128,
    np.dtype(np.float16): DT_HALF, np.dtype(np.uint32): DT_UINT32, np.dtype(np.uint64): DT_UINT64,
    np.dtype(np.object_): DT_STRING,
}
DT_NAMES = {v.number: v.name for v in tf.DataType.values}


class TensorError(ValueError):
    """Malformed or inconsistent tensor (maps to INVALID_ARGUMENT)."""


def np_dtype(dt: int):
    try:
        return DT_TO_NP[dt]
    except KeyError:
        raise TensorError(f"unsupported dtype {DT_NAMES.get(dt, dt)}") from None


def dt_of(arr: np.ndarray) -> int:
    if arr.dtype.kind in ("S", "U", "O"):
        return DT_STRING
    try:
        return NP_TO_DT[arr.dtype]
    except KeyError:
        raise TensorError(f"unsupported numpy dtype {arr.dtype}") from None


def _fill(values: np.ndarray, shape: Tuple[int, ...], dtype) -> np.ndarray:
    n = int(np.prod(shape)) if shape else 1
    if values.size == n:
        return values.reshape(shape)
    if values.size == 0:
        return np.zeros(shape, dtype=dtype)
    if values.size < n:
        out = np.empty(n, dtype=dtype)
        out[: values.size] = values
        out[values.size:] = values[-1]
        return out.reshape(shape)
    raise TensorError(f"tensor has {values.size} values but shape {list(shape)} holds {n}")


def _check_shape(shape: Sequence[int]) -> Tuple[int, ...]:
    for d in shape:
        if d < 0:
            raise TensorError(f"tensor shape {list(shape)} has an unknown (negative) dimension")
    return tuple(int(d) for d in shape)


def make_array_from_native(entry, buf) -> np.ndarray:
    """Build an ndarray from one `_C.parse_predict_request` input tuple.

    Numeric payloads that are raw on the wire are returned as zero-copy views
    into ``buf`` (read-only)."""
    _alias, dt, shape, _unk, storage, off, nbytes, count, owned, strs = entry
    shape = _check_shape(shape)
    if dt == DT_STRING:
        vals = np.empty(len(strs or []), dtype=object)
        if strs:
            vals[:] = strs
        return _fill(vals, shape, object)
    npdt = np_dtype(dt)
    if storage == 1:
        vals = np.frombuffer(buf, dtype=npdt, count=count, offset=off)
    elif storage == 2:
        vals = np.frombuffer(owned, dtype=npdt if dt != DT_BOOL else np.uint8)
        if dt == DT_BOOL:
            vals = vals.astype(np.bool_)
    else:
        vals = np.empty(0, dtype=npdt)
    return _fill(vals, shape, npdt)


def tensor_proto_to_numpy(t) -> np.ndarray:
    """upb TensorProto -> ndarray (control-plane path; hot path uses _C)."""
    from .. import native
    return native.decode_tensor_proto(t.SerializeToString())


def numpy_to_tensor_proto(arr, dtype: Optional[int] = None, use_tensor_content: bool = False):
    """ndarray (or python scalar/list) -> upb TensorProto."""
    from .. import native
    a = np.asarray(arr)
    msg = tf.TensorProto()
    msg.ParseFromString(native.encode_tensor_proto(a, dtype, use_tensor_content))
    return msg


def shape_list(t) -> List[int]:
    return [d.size for d in t.tensor_shape.dim]
