"""``half_plus_two``: the TF-Serving plumbing test model (BASELINE config 1).

y = a*x + b with a = 0.5, b = 2.0 (and y3 = a*x2 + c, c = 3.0).  Inputs arrive
either as a dense float tensor fed straight into ``x`` (Predict) or as
serialized tf.Examples parsed by a ``ParseExample`` node (Classify / Regress /
MultiInference) — the same graph shape TF-Serving's own test export has, so
every RPC of the wire contract can be exercised on it.
"""
from __future__ import annotations

import numpy as np

from ..graph.builder import (CLASSIFY_METHOD, PREDICT_METHOD, REGRESS_METHOD, DType, GraphBuilder,
                             Shape, signature, tensor_info)
from ..savedmodel.saved_model import write_saved_model
from ..utils import tensors as T


def build_graph():
    g = GraphBuilder()
    ser = g.placeholder("tf_example", T.DT_STRING, [-1])
    names = g.const("ParseExample/names", np.array([], dtype=object), T.DT_STRING)
    k_x = g.const("ParseExample/key_x", np.array(b"x", dtype=object), T.DT_STRING)
    k_x2 = g.const("ParseExample/key_x2", np.array(b"x2", dtype=object), T.DT_STRING)
    d_x = g.const("ParseExample/default_x", np.zeros([0], np.float32))
    d_x2 = g.const("ParseExample/default_x2", np.zeros([1], np.float32))
    pe = g.node("ParseExample", "ParseExample/ParseExample", [ser, names, k_x, k_x2, d_x, d_x2],
                Nsparse=0, Ndense=2, sparse_types=[], Tdense=[DType(T.DT_FLOAT), DType(T.DT_FLOAT)],
                dense_shapes=[Shape([1]), Shape([1])])
    x = g.node("Identity", "x", [pe], T=DType(T.DT_FLOAT))
    x2 = g.node("Identity", "x2", [pe + ":1"], T=DType(T.DT_FLOAT))
    a = g.variable("a", np.array(0.5, np.float32))
    b = g.variable("b", np.array(2.0, np.float32))
    c = g.variable("c", np.array(3.0, np.float32))
    ax = g.node("Mul", "Mul", [a, x], T=DType(T.DT_FLOAT))
    y = g.node("AddV2", "y", [ax, b], T=DType(T.DT_FLOAT))
    ax2 = g.node("Mul", "Mul_1", [a, x2], T=DType(T.DT_FLOAT))
    y3 = g.node("AddV2", "y3", [ax2, c], T=DType(T.DT_FLOAT))
    saver = g.add_saver()
    ti_ex = tensor_info(ser, T.DT_STRING, [-1])
    ti_x = tensor_info(x, T.DT_FLOAT, [-1, 1])
    ti_y = tensor_info(y, T.DT_FLOAT, [-1, 1])
    ti_x2 = tensor_info(x2, T.DT_FLOAT, [-1, 1])
    ti_y3 = tensor_info(y3, T.DT_FLOAT, [-1, 1])
    sigs = {
        "serving_default": signature({"x": ti_x}, {"y": ti_y}, PREDICT_METHOD),
        "classify_x_to_y": signature({"inputs": ti_ex}, {"scores": ti_y}, CLASSIFY_METHOD),
        "regress_x_to_y": signature({"inputs": ti_ex}, {"outputs": ti_y}, REGRESS_METHOD),
        "regress_x2_to_y3": signature({"inputs": ti_ex}, {"outputs": ti_y3}, REGRESS_METHOD),
        "classify_x2_to_y3": signature({"inputs": ti_ex}, {"scores": ti_y3}, CLASSIFY_METHOD),
        "predict_x2_to_y3": signature({"x2": ti_x2}, {"y3": ti_y3}, PREDICT_METHOD),
    }
    return g, sigs, saver


def export(export_dir: str) -> str:
    g, sigs, saver = build_graph()
    return write_saved_model(export_dir, g.graph, sigs, g.variables, g.var_dtypes, saver)
