"""TensorBundle (LevelDB table + data shard) and SavedModel I/O."""
import os

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import native
from rust_tensorflow_serving2_amd.savedmodel import bundle as B
from rust_tensorflow_serving2_amd.savedmodel import saved_model as sm
from rust_tensorflow_serving2_amd.utils import tensors as T


def test_sstable_roundtrip_many_blocks():
    kvs = [(b"", b"header")] + [(f"k{i:06d}".encode(), os.urandom(i % 50)) for i in range(3000)]
    data = native.sstable_build(kvs, 4096)
    assert native.sstable_read(data) == kvs


def test_sstable_rejects_unsorted_and_corrupt():
    with pytest.raises(native.WireError):
        native.sstable_build([(b"b", b""), (b"a", b"")])
    data = bytearray(native.sstable_build([(b"a", b"1" * 100)]))
    data[10] ^= 0xFF
    with pytest.raises(native.WireError):
        native.sstable_read(bytes(data))


def test_bundle_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    ts = {"w/kernel": rng.standard_normal((3, 4)).astype(np.float32),
          "b": np.arange(5, dtype=np.int64), "scalar": np.array(2.5, np.float32),
          "bf": np.array([1, 2, 3], np.uint16)}
    prefix = str(tmp_path / "variables" / "variables")
    B.write_bundle(prefix, ts, {"bf": T.DT_BFLOAT16})
    rb = B.Bundle(prefix)
    assert sorted(rb.keys()) == sorted(ts)
    for k, v in ts.items():
        np.testing.assert_array_equal(rb[k], v)
    assert rb.dtype("bf") == T.DT_BFLOAT16


def test_bundle_checksum_detects_corruption(tmp_path):
    prefix = str(tmp_path / "v")
    B.write_bundle(prefix, {"x": np.ones(100, np.float32)})
    path = B.data_file(prefix, 0, 1)
    raw = bytearray(open(path, "rb").read())
    raw[17] ^= 1
    open(path, "wb").write(bytes(raw))
    with pytest.raises(B.DataLossError):
        B.Bundle(prefix)["x"]


def test_saved_model_load(hpt_path):
    b = sm.load(os.path.join(hpt_path, "1"))
    assert b.tags == ["serve"]
    assert b.signatures["serving_default"].method_name == "tensorflow/serving/predict"
    assert float(b.bundle["a"]) == 0.5
    with pytest.raises(sm.SavedModelError):
        sm.load(os.path.join(hpt_path, "1"), tags=("gpu",))
