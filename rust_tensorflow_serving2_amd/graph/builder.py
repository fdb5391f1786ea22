"""Programmatic ``GraphDef`` construction (TF1 graph conventions).

Used by the synthetic exporters (``models/*``) to write real SavedModels —
``Placeholder`` inputs, ``VariableV2`` + ``<var>/read`` Identity weights backed
by a TensorBundle, a ``save/`` Saver subgraph (SaveV2 / RestoreV2 / Assign)
with a matching ``SaverDef`` — the same node vocabulary TF1's official model
exports use (what the reference downloads in ``serving/fetch.sh:7-26``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Union

import numpy as np

from .. import native
from ..schema import tf
from ..utils import tensors as T


class DType(int):
    """Marker so an int attr is encoded as AttrValue.type."""


class Shape(tuple):
    """Marker so a tuple attr is encoded as AttrValue.shape (-1 = unknown dim)."""


def attr_value(v) -> "tf.AttrValue":
    a = tf.AttrValue()
    if isinstance(v, tf.AttrValue):
        a.CopyFrom(v)
    elif isinstance(v, tf.NameAttrList):
        a.func.CopyFrom(v)
    elif isinstance(v, DType):
        a.type = int(v)
    elif isinstance(v, Shape):
        for d in v:
            a.shape.dim.add(size=int(d))
    elif isinstance(v, bool):
        a.b = v
    elif isinstance(v, int):
        a.i = v
    elif isinstance(v, float):
        a.f = v
    elif isinstance(v, (str, bytes)):
        a.s = v.encode() if isinstance(v, str) else v
    elif isinstance(v, np.ndarray):
        a.tensor.ParseFromString(native.encode_tensor_proto(v, None, use_tensor_content=v.dtype != object))
    elif isinstance(v, (list, tuple)):
        lv = a.list
        if all(isinstance(x, DType) for x in v) and v:
            lv.type.extend(int(x) for x in v)
        elif all(isinstance(x, bool) for x in v) and v:
            lv.b.extend(v)
        elif all(isinstance(x, int) for x in v):
            lv.i.extend(v)
        elif all(isinstance(x, float) for x in v):
            lv.f.extend(v)
        elif all(isinstance(x, (str, bytes)) for x in v):
            lv.s.extend(x.encode() if isinstance(x, str) else x for x in v)
        elif all(isinstance(x, Shape) for x in v):
            for s in v:
                sp = lv.shape.add()
                for d in s:
                    sp.dim.add(size=int(d))
        else:
            raise TypeError(f"unsupported list attr {v!r}")
    else:
        raise TypeError(f"unsupported attr value {v!r}")
    return a


class GraphBuilder:
    def __init__(self, producer: int = 27):
        self.graph = tf.GraphDef()
        self.graph.versions.producer = producer
        self._names = set()
        self.variables: Dict[str, np.ndarray] = {}
        self.var_dtypes: Dict[str, int] = {}
        self._scopes: List[str] = []

    # ------------------------------------------------------------ naming
    def scope(self, name: str):
        b = self

        class _S:
            def __enter__(self_):
                b._scopes.append(name)

            def __exit__(self_, *a):
                b._scopes.pop()
        return _S()

    def unique(self, name: str) -> str:
        full = "/".join(self._scopes + [name]) if self._scopes else name
        if full not in self._names:
            self._names.add(full)
            return full
        i = 1
        while f"{full}_{i}" in self._names:
            i += 1
        self._names.add(f"{full}_{i}")
        return f"{full}_{i}"

    # ------------------------------------------------------------ nodes
    def node(self, op: str, name: str, inputs: Sequence[str] = (), **attrs) -> str:
        nd = self.graph.node.add(op=op, name=self.unique(name))
        nd.input.extend(inputs)
        for k, v in attrs.items():
            if v is None:
                continue
            nd.attr[k].CopyFrom(attr_value(v))
        return nd.name

    def placeholder(self, name: str, dtype: int, shape: Sequence[int]) -> str:
        return self.node("Placeholder", name, dtype=DType(dtype), shape=Shape(shape))

    def const(self, name: str, value, dtype: Optional[int] = None) -> str:
        a = np.asarray(value)
        if dtype is None:
            dtype = T.dt_of(a)
        return self.node("Const", name, dtype=DType(dtype), value=a)

    def variable(self, name: str, value: np.ndarray, dtype: Optional[int] = None,
                 resource: bool = False) -> str:
        """Create a checkpointed variable; returns the tensor to read it from."""
        value = np.asarray(value)
        dt = dtype if dtype is not None else T.dt_of(value)
        if resource:
            h = self.node("VarHandleOp", name, dtype=DType(dt), shape=Shape(value.shape),
                          shared_name=("/".join(self._scopes + [name]) if self._scopes else name),
                          container="")
            self.variables[h] = value
            self.var_dtypes[h] = dt
            return self.node("ReadVariableOp", name + "/Read/ReadVariableOp", [h], dtype=DType(dt))
        v = self.node("VariableV2", name, dtype=DType(dt), shape=Shape(value.shape),
                      container="", shared_name="")
        self.variables[v] = value
        self.var_dtypes[v] = dt
        # "<var>/read" is the TF1 convention; bypass scope prefixing (already in v)
        saved = self._scopes
        self._scopes = []
        try:
            r = self.node("Identity", f"{v}/read", [v], T=DType(dt))
        finally:
            self._scopes = saved
        return r

    # ------------------------------------------------------------ saver
    def add_saver(self) -> "tf.SaverDef":
        """TF1 Saver subgraph: save/Const (prefix) -> SaveV2 / RestoreV2 + Assign."""
        saved = self._scopes
        self._scopes = []
        try:
            names = sorted(self.variables, key=lambda s: s.encode())
            prefix = self.node("Const", "save/Const", dtype=DType(T.DT_STRING),
                               value=np.array(b"model", dtype=object))
            tnames = self.node("Const", "save/SaveV2/tensor_names", dtype=DType(T.DT_STRING),
                               value=np.array([n.encode() for n in names], dtype=object))
            slices = self.node("Const", "save/SaveV2/shape_and_slices", dtype=DType(T.DT_STRING),
                               value=np.array([b""] * len(names), dtype=object))
            dts = [DType(self.var_dtypes[n]) for n in names]
            save = self.node("SaveV2", "save/SaveV2", [prefix, tnames, slices] + names, dtypes=dts)
            ctrl = self.node("Identity", "save/control_dependency", [prefix, "^" + save],
                             T=DType(T.DT_STRING))
            rnames = self.node("Const", "save/RestoreV2/tensor_names", dtype=DType(T.DT_STRING),
                               value=np.array([n.encode() for n in names], dtype=object))
            rslices = self.node("Const", "save/RestoreV2/shape_and_slices", dtype=DType(T.DT_STRING),
                                value=np.array([b""] * len(names), dtype=object))
            restore = self.node("RestoreV2", "save/RestoreV2", [prefix, rnames, rslices], dtypes=dts)
            assigns = []
            for i, n in enumerate(names):
                src = restore if i == 0 else f"{restore}:{i}"
                assigns.append(self.node("Assign", "save/Assign", [n, src], T=dts[i],
                                         use_locking=True, validate_shape=True))
            restore_all = self.node("NoOp", "save/restore_all", ["^" + a for a in assigns])
        finally:
            self._scopes = saved
        sd = tf.SaverDef(filename_tensor_name=prefix + ":0", save_tensor_name=ctrl + ":0",
                         restore_op_name=restore_all, max_to_keep=5, sharded=False,
                         keep_checkpoint_every_n_hours=10000.0, version=tf.SaverDef.V2)
        return sd


def tensor_info(name: str, dtype: int, shape: Sequence[int]) -> "tf.TensorInfo":
    ti = tf.TensorInfo(name=name if ":" in name else name + ":0", dtype=dtype)
    for d in shape:
        ti.tensor_shape.dim.add(size=int(d))
    return ti


def signature(inputs: Dict[str, "tf.TensorInfo"], outputs: Dict[str, "tf.TensorInfo"],
              method_name: str) -> "tf.SignatureDef":
    sd = tf.SignatureDef(method_name=method_name)
    for k, v in inputs.items():
        sd.inputs[k].CopyFrom(v)
    for k, v in outputs.items():
        sd.outputs[k].CopyFrom(v)
    return sd


PREDICT_METHOD = "tensorflow/serving/predict"
CLASSIFY_METHOD = "tensorflow/serving/classify"
REGRESS_METHOD = "tensorflow/serving/regress"
