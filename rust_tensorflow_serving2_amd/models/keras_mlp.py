"""A TF2-layout SavedModel (what ``tf.saved_model.save`` of a Keras model writes),
synthesised without TensorFlow: a 2-layer MLP classifier.

Layout reproduced (TF2 object-based SavedModel):

* the serving signature is a ``StatefulPartitionedCall`` of
  ``__inference_signature_wrapper_*``, which calls the model's
  ``__inference_call_*`` function; variables are ``VarHandleOp`` resources
  passed as call arguments and read with ``ReadVariableOp`` inside the body;
* checkpoint keys are object paths
  (``layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE``) that match
  neither node names nor ``shared_name``: the only link is the restore
  function (``__inference__traced_restore_*``: ``RestoreV2`` ->
  ``AssignVariableOp``) called by the ``saver_def.restore_op_name`` node.

Serves as the fixture for TF2 function inlining + saver-graph variable binding
(graph/ir.py ``inline_functions`` / ``restore_keys``).
"""
from __future__ import annotations

import numpy as np

from ..graph.builder import DType, PREDICT_METHOD, Shape, attr_value, signature, tensor_info
from ..savedmodel.saved_model import write_saved_model
from ..schema import tf
from ..utils import tensors as T

KEYS = ["layer_with_weights-0/kernel/.ATTRIBUTES/VARIABLE_VALUE",
        "layer_with_weights-0/bias/.ATTRIBUTES/VARIABLE_VALUE",
        "layer_with_weights-1/kernel/.ATTRIBUTES/VARIABLE_VALUE",
        "layer_with_weights-1/bias/.ATTRIBUTES/VARIABLE_VALUE"]
VARS = ["dense/kernel", "dense/bias", "dense_1/kernel", "dense_1/bias"]


def _fn_node(fdef, op, name, inputs, **attrs):
    nd = fdef.node_def.add(op=op, name=name)
    nd.input.extend(inputs)
    for k, v in attrs.items():
        nd.attr[k].CopyFrom(attr_value(v))
    return nd


def _args(fdef, names_types):
    for n, t in names_types:
        fdef.signature.input_arg.add(name=n, type=t)


def weights(d_in: int = 16, hidden: int = 32, classes: int = 5, seed: int = 0):
    rng = np.random.default_rng(seed)
    return [(rng.standard_normal((d_in, hidden)) / np.sqrt(d_in)).astype(np.float32),
            (rng.standard_normal(hidden) * 0.1).astype(np.float32),
            (rng.standard_normal((hidden, classes)) / np.sqrt(hidden)).astype(np.float32),
            (rng.standard_normal(classes) * 0.1).astype(np.float32)]


def reference(x: np.ndarray, w) -> np.ndarray:
    h = np.maximum(x @ w[0] + w[1], 0)
    z = h @ w[2] + w[3]
    e = np.exp(z - z.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def build(d_in: int = 16, hidden: int = 32, classes: int = 5, seed: int = 0):
    w = weights(d_in, hidden, classes, seed)
    F, R = T.DT_FLOAT, 20   # DT_RESOURCE
    gd = tf.GraphDef()
    lib = gd.library

    call = lib.function.add()
    call.signature.name = "__inference_call_1024"
    _args(call, [("inputs", F)] + [(f"{v.replace('/', '_')}_readvariableop_resource", R) for v in VARS])
    call.signature.output_arg.add(name="identity", type=F)
    res = [a.name for a in call.signature.input_arg[1:]]
    for i, (rname, vn) in enumerate(zip(res, VARS)):
        _fn_node(call, "ReadVariableOp", f"{vn.replace('/', '_')}/ReadVariableOp", [rname], dtype=DType(F))
    _fn_node(call, "MatMul", "dense/MatMul", ["inputs", "dense_kernel/ReadVariableOp:value:0"], T=DType(F),
             transpose_a=False, transpose_b=False)
    _fn_node(call, "BiasAdd", "dense/BiasAdd", ["dense/MatMul:product:0", "dense_bias/ReadVariableOp:value:0"],
             T=DType(F))
    _fn_node(call, "Relu", "dense/Relu", ["dense/BiasAdd:output:0"], T=DType(F))
    _fn_node(call, "MatMul", "dense_1/MatMul", ["dense/Relu:activations:0", "dense_1_kernel/ReadVariableOp:value:0"],
             T=DType(F), transpose_a=False, transpose_b=False)
    _fn_node(call, "BiasAdd", "dense_1/BiasAdd",
             ["dense_1/MatMul:product:0", "dense_1_bias/ReadVariableOp:value:0"], T=DType(F))
    _fn_node(call, "Softmax", "dense_1/Softmax", ["dense_1/BiasAdd:output:0"], T=DType(F))
    _fn_node(call, "Identity", "Identity", ["dense_1/Softmax:softmax:0", "^dense_kernel/ReadVariableOp"], T=DType(F))
    call.ret["identity"] = "Identity:output:0"

    wrap = lib.function.add()
    wrap.signature.name = "__inference_signature_wrapper_2048"
    _args(wrap, [("x", F)] + [(f"unknown_{i}", R) for i in range(4)])
    wrap.signature.output_arg.add(name="output_0", type=F)
    _fn_node(wrap, "StatefulPartitionedCall", "StatefulPartitionedCall",
             ["x"] + [f"unknown_{i}" for i in range(4)], Tin=[DType(F)] + [DType(R)] * 4, Tout=[DType(F)],
             f=tf.NameAttrList(name=call.signature.name))
    _fn_node(wrap, "Identity", "Identity", ["StatefulPartitionedCall:output:0"], T=DType(F))
    wrap.ret["output_0"] = "Identity:output:0"

    rest = lib.function.add()
    rest.signature.name = "__inference__traced_restore_4096"
    _args(rest, [("file_prefix", T.DT_STRING)] + [(f"assignvariableop_{i}_resource", R) for i in range(4)])
    rest.signature.output_arg.add(name="identity_5", type=T.DT_STRING)
    _fn_node(rest, "Const", "RestoreV2/tensor_names", [], dtype=DType(T.DT_STRING),
             value=np.array([k.encode() for k in KEYS], dtype=object))
    _fn_node(rest, "Const", "RestoreV2/shape_and_slices", [], dtype=DType(T.DT_STRING),
             value=np.array([b""] * 4, dtype=object))
    _fn_node(rest, "RestoreV2", "RestoreV2",
             ["file_prefix", "RestoreV2/tensor_names:output:0", "RestoreV2/shape_and_slices:output:0"],
             dtypes=[DType(F)] * 4)
    for i in range(4):
        _fn_node(rest, "Identity", f"Identity_{i}", [f"RestoreV2:tensors:{i}"], T=DType(F))
        _fn_node(rest, "AssignVariableOp", f"AssignVariableOp_{i}",
                 [f"assignvariableop_{i}_resource", f"Identity_{i}:output:0"], dtype=DType(F))
    _fn_node(rest, "NoOp", "NoOp", [f"^AssignVariableOp_{i}" for i in range(4)])
    _fn_node(rest, "Identity", "Identity_5", ["file_prefix", "^NoOp"], T=DType(T.DT_STRING))
    rest.ret["identity_5"] = "Identity_5:output:0"

    def node(op, name, inputs=(), **attrs):
        nd = gd.node.add(op=op, name=name)
        nd.input.extend(inputs)
        for k, v in attrs.items():
            nd.attr[k].CopyFrom(attr_value(v))
        return name

    x = node("Placeholder", "serving_default_x", dtype=DType(F), shape=Shape((-1, d_in)))
    handles = [node("VarHandleOp", vn, dtype=DType(F), shape=Shape(a.shape), shared_name=vn, container="")
               for vn, a in zip(VARS, w)]
    node("StatefulPartitionedCall", "StatefulPartitionedCall", [x] + handles, Tin=[DType(F)] + [DType(R)] * 4,
         Tout=[DType(F)], f=tf.NameAttrList(name=wrap.signature.name))
    fname = node("Placeholder", "saver_filename", dtype=DType(T.DT_STRING), shape=Shape(()))
    node("StatefulPartitionedCall", "StatefulPartitionedCall_2", [fname] + handles,
         Tin=[DType(T.DT_STRING)] + [DType(R)] * 4, Tout=[DType(T.DT_STRING)],
         f=tf.NameAttrList(name=rest.signature.name))
    sigs = {"serving_default": signature({"x": tensor_info(x, F, (-1, d_in))},
                                         {"output_0": tensor_info("StatefulPartitionedCall", F, (-1, classes))},
                                         PREDICT_METHOD)}
    saver = tf.SaverDef(filename_tensor_name="saver_filename:0", save_tensor_name="StatefulPartitionedCall_1:0",
                        restore_op_name="StatefulPartitionedCall_2", version=tf.SaverDef.V2)
    variables = dict(zip(KEYS, w))
    return gd, sigs, variables, saver, w


def export(export_dir: str, **kw) -> str:
    gd, sigs, variables, saver, _w = build(**kw)
    return write_saved_model(export_dir, gd, sigs, variables, {k: T.DT_FLOAT for k in variables}, saver)
