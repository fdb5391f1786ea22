"""TensorBundle (TF checkpoint V2) reader/writer.

``<prefix>.index`` is a LevelDB table (native ``_C.sstable_*``) whose empty key
holds a ``BundleHeaderProto`` and every other key (a variable name, sorted)
a ``BundleEntryProto`` locating the tensor bytes inside
``<prefix>.data-<shard>-of-<num_shards>``.  Data shards are mmap'd (never
slurped), so tensors come back as zero-copy read-only views; each tensor's
masked crc32c is verified (``DataLossError`` on mismatch) before it is used.

This is the ``variables/`` half of the SavedModel layout the reference's
fixture ships (``serving/fetch.sh:22-26``: ``models/1/{saved_model.pb,variables}``).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional

import numpy as np

from .. import native
from ..schema import tf
from ..utils import tensors as T


class DataLossError(IOError):
    """Corrupt checkpoint bytes (maps to DATA_LOSS)."""


def data_file(prefix: str, shard: int, num_shards: int) -> str:
    return f"{prefix}.data-{shard:05d}-of-{num_shards:05d}"


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray],
                 dtypes: Optional[Dict[str, int]] = None) -> None:
    """Write one-shard bundle.  ``dtypes`` overrides the inferred DataType
    (e.g. DT_BFLOAT16 for uint16-bit arrays)."""
    dtypes = dtypes or {}
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    names = sorted(tensors, key=lambda s: s.encode())
    kvs = []
    off = 0
    with open(data_file(prefix, 0, 1), "wb") as f:
        for name in names:
            a = np.asarray(tensors[name])
            dt = dtypes.get(name) or T.dt_of(a)
            if dt == T.DT_STRING:
                raise ValueError("string variables are not supported in bundles")
            if dt == T.DT_BFLOAT16:
                if a.dtype.itemsize != 2:
                    raise ValueError(f"{name}: DT_BFLOAT16 needs the raw 16-bit pattern (got {a.dtype})")
            else:
                want = np.dtype(T.np_dtype(dt))
                if a.dtype != want:
                    a = a.astype(want)      # the entry's bytes must match its declared dtype
            a = np.require(a, requirements="C")
            raw = memoryview(a.reshape(-1)).cast("B") if a.size else b""
            f.write(raw)
            e = tf.BundleEntryProto(dtype=dt, shard_id=0, offset=off, size=len(raw),
                                    crc32c=native.crc32c_mask(native.crc32c(raw)))
            for d in a.shape:
                e.shape.dim.add(size=int(d))
            kvs.append((name.encode(), e.SerializeToString()))
            off += len(raw)
    header = tf.BundleHeaderProto(num_shards=1, endianness=tf.BundleHeaderProto.LITTLE)
    header.version.producer = 1
    kvs.insert(0, (b"", header.SerializeToString()))
    tmp = prefix + ".index.tmp"
    with open(tmp, "wb") as f:
        f.write(native.sstable_build(kvs))
    os.replace(tmp, prefix + ".index")


class Bundle:
    """Read side.  ``Bundle(prefix)[name]`` -> ndarray view (bf16 as uint16)."""

    def __init__(self, prefix: str, verify: bool = True):
        self.prefix = prefix
        self.verify = verify
        with open(prefix + ".index", "rb") as f:
            raw = f.read()
        try:
            kvs = native.sstable_read(raw, verify)
        except native.WireError as e:
            raise DataLossError(f"{prefix}.index: {e}") from None
        if not kvs or kvs[0][0] != b"":
            raise DataLossError(f"{prefix}.index: missing bundle header")
        self.header = tf.BundleHeaderProto.FromString(kvs[0][1])
        if self.header.endianness != tf.BundleHeaderProto.LITTLE:
            raise DataLossError("big-endian bundles are not supported")
        self.entries: Dict[str, object] = {}
        for k, v in kvs[1:]:
            self.entries[k.decode()] = tf.BundleEntryProto.FromString(v)
        n = max(1, self.header.num_shards)
        self._shards = {}
        self._n = n
        self._verified = set()

    def _shard(self, i: int):
        if i not in self._shards:
            path = data_file(self.prefix, i, self._n)
            self._shards[i] = native.MappedFile(path)
        return self._shards[i]

    def keys(self) -> Iterable[str]:
        return self.entries.keys()

    def __contains__(self, name: str) -> bool:
        return name in self.entries

    def dtype(self, name: str) -> int:
        return self.entries[name].dtype

    def shape(self, name: str):
        return tuple(d.size for d in self.entries[name].shape.dim)

    def __getitem__(self, name: str) -> np.ndarray:
        e = self.entries[name]
        if e.slices:
            raise ValueError(f"{name}: partitioned (sliced) variables are not supported")
        shard = self._shard(e.shard_id)
        if e.offset + e.size > len(shard):
            raise DataLossError(f"{name}: entry points past the end of its data shard")
        if self.verify and name not in self._verified:
            if native.crc32c_mask(shard.crc32c(e.offset, e.size)) != e.crc32c:
                raise DataLossError(f"{name}: checksum mismatch in {self.prefix}")
            self._verified.add(name)
        npdt = T.np_dtype(e.dtype)
        shape = tuple(d.size for d in e.shape.dim)
        count = int(np.prod(shape)) if shape else 1
        buf = np.frombuffer(shard, dtype=np.uint8, count=e.size, offset=e.offset)
        arr = buf.view(npdt if e.dtype != T.DT_BOOL else np.uint8)
        if arr.size != count:
            raise DataLossError(f"{name}: size {e.size} does not match shape {list(shape)}")
        if e.dtype == T.DT_BOOL:
            arr = arr.astype(np.bool_)
        return arr.reshape(shape)
