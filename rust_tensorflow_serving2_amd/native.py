"""Python face of the native CPU data plane (``_C``).

Fails loudly when the extension is missing: run
``python -m rust_tensorflow_serving2_amd._build`` (or ``__graft_entry__.build()``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

try:
    from . import _C  # noqa: F401
except ImportError as e:  # pragma: no cover - exercised only on a broken build
    raise ImportError(
        "rust_tensorflow_serving2_amd._C is not built; run "
        "`python -m rust_tensorflow_serving2_amd._build`") from e

from .utils import tensors as T

WireError = _C.WireError
crc32c = _C.crc32c
crc32c_mask = _C.crc32c_mask
crc32c_unmask = _C.crc32c_unmask


def spec_tuple(name: str, version: Optional[int] = None, label: Optional[str] = None,
               signature_name: str = "") -> tuple:
    return (name.encode(), version, None if label is None else label.encode(), signature_name.encode())


def _out_entry(alias: str, arr, dtype: Optional[int] = None):
    a = np.asarray(arr)
    dt = dtype if dtype is not None else T.dt_of(a)
    if dt == T.DT_STRING:
        flat = [x if isinstance(x, (bytes, bytearray)) else str(x).encode() for x in a.reshape(-1).tolist()]
        return (alias.encode(), dt, list(a.shape), flat)
    if dt == T.DT_BOOL:
        a = a.astype(np.uint8)
    elif dt in (T.DT_BFLOAT16,):
        a = a.view(np.uint16) if a.dtype.itemsize == 2 else a
    else:
        want = np.dtype(T.np_dtype(dt))
        if a.dtype != want:
            a = a.astype(want)
    shape = list(a.shape)
    a = np.require(a, requirements="C")   # (ascontiguousarray would turn 0-d into 1-d)
    return (alias.encode(), dt, shape, a.reshape(-1).view(np.uint8) if a.size else np.zeros(0, np.uint8))


def encode_predict_response(spec: Optional[tuple], outputs: Dict[str, np.ndarray],
                            dtypes: Optional[Dict[str, int]] = None,
                            use_tensor_content: bool = False) -> bytes:
    dtypes = dtypes or {}
    return _C.encode_predict_response(
        spec, [_out_entry(k, v, dtypes.get(k)) for k, v in outputs.items()], use_tensor_content)


def encode_predict_request(spec: tuple, inputs: Dict[str, np.ndarray], output_filter: Sequence[str] = (),
                           dtypes: Optional[Dict[str, int]] = None, use_tensor_content: bool = False) -> bytes:
    dtypes = dtypes or {}
    return _C.encode_predict_request(
        spec, [_out_entry(k, v, dtypes.get(k)) for k, v in inputs.items()],
        [f.encode() for f in output_filter], use_tensor_content)


def decode_predict_request(buf) -> Tuple[Optional[tuple], Dict[str, np.ndarray], List[str], Dict[str, int]]:
    """-> (spec, {alias: ndarray}, output_filter, {alias: dtype}).  Arrays may be
    zero-copy views into ``buf``."""
    spec, entries, filt = _C.parse_predict_request(buf)
    arrays, dts = {}, {}
    for e in entries:
        alias = e[0].decode()
        arrays[alias] = T.make_array_from_native(e, buf)
        dts[alias] = e[1]
    return spec, arrays, [f.decode() for f in filt], dts


def encode_tensor_proto(arr, dtype: Optional[int] = None, use_tensor_content: bool = False) -> bytes:
    """ndarray -> serialized TensorProto (via a one-entry PredictResponse)."""
    resp = encode_predict_response(None, {"t": arr}, {"t": dtype} if dtype is not None else None,
                                   use_tensor_content)
    # resp = field1{ key, value } -> extract the value bytes
    from .schema import serving
    r = serving.PredictResponse.FromString(resp)
    return r.outputs["t"].SerializeToString()


def decode_tensor_proto(data: bytes) -> np.ndarray:
    from .schema import serving
    req = serving.PredictRequest()
    req.inputs["t"].ParseFromString(data)
    buf = req.SerializeToString()
    _spec, arrays, _f, _d = decode_predict_request(buf)
    return np.array(arrays["t"])  # own the memory


MappedFile = _C.MappedFile
sstable_build = _C.sstable_build
sstable_read = _C.sstable_read


def encode_image_request(spec: tuple, alias: str, pixels: np.ndarray, dims, lut: np.ndarray) -> bytes:
    """PredictRequest with one DT_FLOAT ``float_val`` tensor: ``lut[pixels]``
    (u8 -> f32 through a 256-entry table) with shape ``dims`` (C++)."""
    return _C.encode_image_request(spec, alias, np.ascontiguousarray(pixels, dtype=np.uint8).reshape(-1),
                                   [int(d) for d in dims], np.ascontiguousarray(lut, dtype=np.float32))
