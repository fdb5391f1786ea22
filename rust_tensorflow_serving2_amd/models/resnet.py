"""ResNet-50 (v1.5 and v2) SavedModel exporter with random-init weights.

The graph follows TF's official NHWC ResNet export — the model the reference
fetches (``serving/fetch.sh:7-9``, ``resnet_v2_fp32_savedmodel_NHWC``):
``input_tensor`` [-1,224,224,3] f32 -> fixed-padding ``Pad`` + ``Conv2D``
(VALID) for strided convs, ``FusedBatchNormV3`` (inference), ``Relu``,
``MaxPool`` 3x3/2 SAME, bottleneck blocks [3,4,6,3] (v1.5: stride on the 3x3;
v2: pre-activation), ``Mean`` over H,W, ``MatMul`` + ``BiasAdd`` to 1001 logits,
``ArgMax`` -> ``classes`` (int64) and ``Softmax`` -> ``probabilities``.
Signatures ``serving_default`` and ``predict`` map alias ``"input"`` (the alias
the Rust client hard-codes, src/lib.rs:256-257) to ``input_tensor:0``.

No network in the sandbox, so weights are random (He-normal convs, mild BN
statistics) and the exported bytes are a genuine TF1 SavedModel.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from ..graph.builder import PREDICT_METHOD, DType, GraphBuilder, Shape, signature, tensor_info
from ..savedmodel.saved_model import write_saved_model
from ..utils import tensors as T

F32 = DType(T.DT_FLOAT)
BLOCKS_50 = (3, 4, 6, 3)
NUM_CLASSES = 1001


class _Init:
    def __init__(self, seed: int):
        self.rng = np.random.default_rng(seed)

    def conv(self, kh, kw, cin, cout):
        std = np.sqrt(2.0 / (kh * kw * cin))
        return (self.rng.standard_normal((kh, kw, cin, cout)) * std).astype(np.float32)

    def bn(self, c, gamma_scale=1.0):
        r = self.rng
        gamma = (gamma_scale * (1.0 + 0.1 * r.standard_normal(c))).astype(np.float32)
        beta = (0.05 * r.standard_normal(c)).astype(np.float32)
        mean = (0.05 * r.standard_normal(c)).astype(np.float32)
        var = (1.0 + 0.1 * np.abs(r.standard_normal(c))).astype(np.float32)
        return gamma, beta, mean, var


def _fixed_pad(g: GraphBuilder, x: str, k: int) -> str:
    pad_total = k - 1
    beg = pad_total // 2
    end = pad_total - beg
    pads = g.const("Pad/paddings", np.array([[0, 0], [beg, end], [beg, end], [0, 0]], np.int32))
    return g.node("Pad", "Pad", [x, pads], T=F32, Tpaddings=DType(T.DT_INT32))


def _conv(g, init, x, k, cin, cout, stride, name):
    with g.scope(name):
        if stride > 1:
            x = _fixed_pad(g, x, k)
            padding = "VALID"
        else:
            padding = "SAME"
        w = g.variable("kernel", init.conv(k, k, cin, cout))
        return g.node("Conv2D", "Conv2D", [x, w], T=F32, strides=[1, stride, stride, 1],
                      padding=padding, data_format="NHWC", dilations=[1, 1, 1, 1],
                      use_cudnn_on_gpu=True, explicit_paddings=[])


def _bn(g, init, x, c, name, gamma_scale=1.0, eps=1e-5):
    with g.scope(name):
        gamma, beta, mean, var = init.bn(c, gamma_scale)
        vg = g.variable("gamma", gamma)
        vb = g.variable("beta", beta)
        vm = g.variable("moving_mean", mean)
        vv = g.variable("moving_variance", var)
        return g.node("FusedBatchNormV3", "FusedBatchNormV3", [x, vg, vb, vm, vv], T=F32, U=F32,
                      epsilon=eps, data_format="NHWC", is_training=False,
                      exponential_avg_factor=1.0)


def _relu(g, x):
    return g.node("Relu", "Relu", [x], T=F32)


def _block_v1(g, init, x, cin, filters, stride, project, name):
    with g.scope(name):
        shortcut = x
        if project:
            s = _conv(g, init, x, 1, cin, 4 * filters, stride, "shortcut_conv")
            shortcut = _bn(g, init, s, 4 * filters, "shortcut_bn")
        y = _relu(g, _bn(g, init, _conv(g, init, x, 1, cin, filters, 1, "conv1"), filters, "bn1"))
        y = _relu(g, _bn(g, init, _conv(g, init, y, 3, filters, filters, stride, "conv2"), filters, "bn2"))
        y = _bn(g, init, _conv(g, init, y, 1, filters, 4 * filters, 1, "conv3"), 4 * filters, "bn3",
                gamma_scale=0.25)
        y = g.node("AddV2", "add", [y, shortcut], T=F32)
        return _relu(g, y)


def _block_v2(g, init, x, cin, filters, stride, project, name):
    with g.scope(name):
        pre = _relu(g, _bn(g, init, x, cin, "preact_bn"))
        shortcut = x
        if project:
            shortcut = _conv(g, init, pre, 1, cin, 4 * filters, stride, "shortcut_conv")
        y = _conv(g, init, pre, 1, cin, filters, 1, "conv1")
        y = _relu(g, _bn(g, init, y, filters, "bn1"))
        y = _conv(g, init, y, 3, filters, filters, stride, "conv2")
        y = _relu(g, _bn(g, init, y, filters, "bn2"))
        y = _conv(g, init, y, 1, filters, 4 * filters, 1, "conv3")
        y = g.node("Mul", "residual_scale", [y, g.const("scale", np.array(0.25, np.float32))], T=F32)
        return g.node("AddV2", "add", [y, shortcut], T=F32)


def build_graph(version: str = "v1.5", blocks=BLOCKS_50, num_classes: int = NUM_CLASSES,
                seed: int = 0, width: int = 64, image_size: int = 224):
    g = GraphBuilder()
    init = _Init(seed)
    x = g.placeholder("input_tensor", T.DT_FLOAT, [-1, image_size, image_size, 3])
    with g.scope("resnet_model"):
        y = _conv(g, init, x, 7, 3, width, 2, "initial_conv")
        if version != "v2":
            y = _relu(g, _bn(g, init, y, width, "initial_bn"))
        y = g.node("MaxPool", "initial_max_pool", [y], T=F32, ksize=[1, 3, 3, 1],
                   strides=[1, 2, 2, 1], padding="SAME", data_format="NHWC")
        cin = width
        block_fn = _block_v2 if version == "v2" else _block_v1
        for si, n in enumerate(blocks):
            filters = width * (2 ** si)
            for bi in range(n):
                stride = 2 if (bi == 0 and si > 0) else 1
                y = block_fn(g, init, y, cin, filters, stride, bi == 0, f"block_layer{si + 1}_{bi}")
                cin = 4 * filters
        if version == "v2":
            y = _relu(g, _bn(g, init, y, cin, "postnorm"))
        axes = g.const("Mean/reduction_indices", np.array([1, 2], np.int32))
        y = g.node("Mean", "Mean", [y, axes], T=F32, Tidx=DType(T.DT_INT32), keep_dims=False)
        with g.scope("dense"):
            w = g.variable("kernel", (init.rng.standard_normal((cin, num_classes)) *
                                      np.sqrt(1.0 / cin)).astype(np.float32))
            b = g.variable("bias", (0.01 * init.rng.standard_normal(num_classes)).astype(np.float32))
            y = g.node("MatMul", "MatMul", [y, w], T=F32, transpose_a=False, transpose_b=False)
            y = g.node("BiasAdd", "BiasAdd", [y, b], T=F32, data_format="NHWC")
    logits = g.node("Identity", "final_dense", [y], T=F32)
    dim = g.const("ArgMax/dimension", np.array(1, np.int32))
    classes = g.node("ArgMax", "ArgMax", [logits, dim], T=F32, Tidx=DType(T.DT_INT32),
                     output_type=DType(T.DT_INT64))
    probs = g.node("Softmax", "softmax_tensor", [logits], T=F32)
    saver = g.add_saver()
    ins = {"input": tensor_info(x, T.DT_FLOAT, [-1, image_size, image_size, 3])}
    outs = {"classes": tensor_info(classes, T.DT_INT64, [-1]),
            "probabilities": tensor_info(probs, T.DT_FLOAT, [-1, num_classes])}
    sig = signature(ins, outs, PREDICT_METHOD)
    return g, {"serving_default": sig, "predict": sig}, saver


def export(export_dir: str, version: str = "v1.5", seed: int = 0, blocks=BLOCKS_50,
           num_classes: int = NUM_CLASSES, width: int = 64, image_size: int = 224) -> str:
    g, sigs, saver = build_graph(version, blocks, num_classes, seed, width, image_size)
    return write_saved_model(export_dir, g.graph, sigs, g.variables, g.var_dtypes, saver)
