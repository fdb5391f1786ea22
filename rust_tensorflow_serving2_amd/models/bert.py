"""BERT (base by default) sequence-classifier SavedModel exporter, random init.

BASELINE config 3 ("BERT-base Predict seq=128 bf16 with dynamic batching").
The graph is written in the op vocabulary of the original TF1 BERT export
(google-research ``modeling.py``): ``GatherV2`` embedding lookups, position
embeddings via ``Slice``, decomposed LayerNorm (``Mean``/``SquaredDifference``/
``Rsqrt``/...), 2-D ``MatMul`` dense layers, per-head ``Reshape``/``Transpose``,
``BatchMatMulV2`` attention with a ``-10000`` additive mask, tanh-approximate
GELU (``Pow``/``Tanh`` subgraph), tanh pooler and a softmax classifier.  The
fusion passes (``graph/patterns.py``) recognise exactly these subgraphs.

Signature ``serving_default`` (predict): inputs ``input_ids``, ``input_mask``,
``segment_ids`` (int32 [-1, S]); outputs ``probabilities`` [-1, num_labels]
and ``pooled_output`` [-1, hidden].
"""
from __future__ import annotations

import math

import numpy as np

from ..graph.builder import PREDICT_METHOD, DType, GraphBuilder, signature, tensor_info
from ..savedmodel.saved_model import write_saved_model
from ..utils import tensors as T

F32 = DType(T.DT_FLOAT)
I32 = DType(T.DT_INT32)


class BertConfig:
    def __init__(self, vocab_size=30522, hidden=768, layers=12, heads=12, intermediate=3072,
                 max_position=512, type_vocab=2, num_labels=2, seq_len=128, eps=1e-12):
        self.vocab_size, self.hidden, self.layers, self.heads = vocab_size, hidden, layers, heads
        self.intermediate, self.max_position, self.type_vocab = intermediate, max_position, type_vocab
        self.num_labels, self.seq_len, self.eps = num_labels, seq_len, eps


BASE = BertConfig()


def _c(g, name, v, dt=None):
    return g.const(name, np.asarray(v, dtype=np.float32 if dt is None else dt))


def layer_norm(g: GraphBuilder, x: str, dim: int, rng, eps: float, name: str) -> str:
    with g.scope(name):
        gamma = g.variable("gamma", (1.0 + 0.05 * rng.standard_normal(dim)).astype(np.float32))
        beta = g.variable("beta", (0.02 * rng.standard_normal(dim)).astype(np.float32))
        axes = g.const("moments/mean/reduction_indices", np.array([-1], np.int32))
        mean = g.node("Mean", "moments/mean", [x, axes], T=F32, Tidx=I32, keep_dims=True)
        sg = g.node("StopGradient", "moments/StopGradient", [mean], T=F32)
        sqd = g.node("SquaredDifference", "moments/SquaredDifference", [x, sg], T=F32)
        axes2 = g.const("moments/variance/reduction_indices", np.array([-1], np.int32))
        var = g.node("Mean", "moments/variance", [sqd, axes2], T=F32, Tidx=I32, keep_dims=True)
        e = _c(g, "batchnorm/add/y", eps)
        add = g.node("AddV2", "batchnorm/add", [var, e], T=F32)
        rs = g.node("Rsqrt", "batchnorm/Rsqrt", [add], T=F32)
        mul = g.node("Mul", "batchnorm/mul", [rs, gamma], T=F32)
        mul1 = g.node("Mul", "batchnorm/mul_1", [x, mul], T=F32)
        mul2 = g.node("Mul", "batchnorm/mul_2", [mean, mul], T=F32)
        sub = g.node("Sub", "batchnorm/sub", [beta, mul2], T=F32)
        return g.node("AddV2", "batchnorm/add_1", [mul1, sub], T=F32)


def dense(g, x, din, dout, rng, name, act=None, std=0.02):
    with g.scope(name):
        w = g.variable("kernel", (rng.standard_normal((din, dout)) * std).astype(np.float32))
        b = g.variable("bias", (0.02 * rng.standard_normal(dout)).astype(np.float32))
        y = g.node("MatMul", "MatMul", [x, w], T=F32, transpose_a=False, transpose_b=False)
        y = g.node("BiasAdd", "BiasAdd", [y, b], T=F32, data_format="NHWC")
        if act == "gelu":
            y = gelu(g, y)
        elif act == "tanh":
            y = g.node("Tanh", "Tanh", [y], T=F32)
        return y


def gelu(g, x):
    """0.5 * x * (1 + tanh(sqrt(2/pi) * (x + 0.044715 x^3)))  (BERT's gelu)."""
    p = g.node("Pow", "Pow", [x, _c(g, "Pow/y", 3.0)], T=F32)
    m = g.node("Mul", "mul", [_c(g, "mul/x", 0.044715), p], T=F32)
    a = g.node("AddV2", "add", [x, m], T=F32)
    m1 = g.node("Mul", "mul_1", [_c(g, "mul_1/x", math.sqrt(2 / math.pi)), a], T=F32)
    t = g.node("Tanh", "Tanh", [m1], T=F32)
    a1 = g.node("AddV2", "add_1", [_c(g, "add_1/x", 1.0), t], T=F32)
    m2 = g.node("Mul", "mul_2", [_c(g, "mul_2/x", 0.5), a1], T=F32)
    return g.node("Mul", "mul_3", [x, m2], T=F32)


def build_graph(cfg: BertConfig = BASE, seed: int = 0):
    g = GraphBuilder()
    rng = np.random.default_rng(seed)
    S, Hd, nH = cfg.seq_len, cfg.hidden, cfg.heads
    dH = Hd // nH
    ids = g.placeholder("input_ids", T.DT_INT32, [-1, S])
    mask = g.placeholder("input_mask", T.DT_INT32, [-1, S])
    seg = g.placeholder("segment_ids", T.DT_INT32, [-1, S])
    with g.scope("bert"):
        with g.scope("embeddings"):
            table = g.variable("word_embeddings", (rng.standard_normal((cfg.vocab_size, Hd)) * 0.02).astype(np.float32))
            flat = g.node("Reshape", "Reshape", [ids, g.const("Reshape/shape", np.array([-1], np.int32))], T=I32)
            emb = g.node("GatherV2", "GatherV2", [table, flat, g.const("GatherV2/axis", np.array(0, np.int32))],
                         Tparams=F32, Tindices=I32, Taxis=I32, batch_dims=0)
            emb = g.node("Reshape", "Reshape_1", [emb, g.const("Reshape_1/shape", np.array([-1, S, Hd], np.int32))],
                         T=F32)
            ttab = g.variable("token_type_embeddings",
                              (rng.standard_normal((cfg.type_vocab, Hd)) * 0.02).astype(np.float32))
            fseg = g.node("Reshape", "Reshape_2", [seg, g.const("Reshape_2/shape", np.array([-1], np.int32))], T=I32)
            temb = g.node("GatherV2", "GatherV2_1", [ttab, fseg, g.const("GatherV2_1/axis", np.array(0, np.int32))],
                          Tparams=F32, Tindices=I32, Taxis=I32, batch_dims=0)
            temb = g.node("Reshape", "Reshape_3", [temb, g.const("Reshape_3/shape", np.array([-1, S, Hd], np.int32))],
                          T=F32)
            emb = g.node("AddV2", "add", [emb, temb], T=F32)
            ptab = g.variable("position_embeddings",
                              (rng.standard_normal((cfg.max_position, Hd)) * 0.02).astype(np.float32))
            pos = g.node("Slice", "Slice", [ptab, g.const("Slice/begin", np.array([0, 0], np.int32)),
                                            g.const("Slice/size", np.array([S, -1], np.int32))], T=F32, Index=I32)
            pos = g.node("Reshape", "Reshape_4", [pos, g.const("Reshape_4/shape", np.array([1, S, Hd], np.int32))],
                         T=F32)
            emb = g.node("AddV2", "add_1", [emb, pos], T=F32)
            emb = layer_norm(g, emb, Hd, rng, cfg.eps, "LayerNorm")
        with g.scope("encoder"):
            m = g.node("Reshape", "Reshape", [mask, g.const("Reshape/shape", np.array([-1, 1, S], np.int32))], T=I32)
            m = g.node("Cast", "Cast", [m], SrcT=I32, DstT=F32, Truncate=False)
            ones = g.const("ones", np.ones((1, S, 1), np.float32))
            m = g.node("Mul", "mul", [ones, m], T=F32)           # [B, S, S]
            x = g.node("Reshape", "Reshape_1", [emb, g.const("Reshape_1/shape", np.array([-1, Hd], np.int32))], T=F32)
            for li in range(cfg.layers):
                with g.scope(f"layer_{li}"):
                    with g.scope("attention"):
                        with g.scope("self"):
                            ex = g.node("ExpandDims", "ExpandDims", [m, g.const("ExpandDims/dim", np.array(1, np.int32))],
                                        T=F32, Tdim=I32)
                            sub = g.node("Sub", "sub", [_c(g, "sub/x", 1.0), ex], T=F32)
                            adder = g.node("Mul", "mul_1", [sub, _c(g, "mul_1/y", -10000.0)], T=F32)
                            heads = []
                            for nm in ("query", "key", "value"):
                                y = dense(g, x, Hd, Hd, rng, nm)
                                y = g.node("Reshape", f"Reshape_{nm}", [y, g.const(f"Reshape_{nm}/shape",
                                                                                    np.array([-1, S, nH, dH], np.int32))],
                                           T=F32)
                                y = g.node("Transpose", f"transpose_{nm}",
                                           [y, g.const(f"transpose_{nm}/perm", np.array([0, 2, 1, 3], np.int32))],
                                           T=F32, Tperm=I32)
                                heads.append(y)
                            q, k, v = heads
                            sc = g.node("BatchMatMulV2", "MatMul", [q, k], T=F32, adj_x=False, adj_y=True)
                            sc = g.node("Mul", "Mul", [sc, _c(g, "Mul/y", 1.0 / math.sqrt(dH))], T=F32)
                            sc = g.node("AddV2", "add", [sc, adder], T=F32)
                            pr = g.node("Softmax", "Softmax", [sc], T=F32)
                            ctx = g.node("BatchMatMulV2", "MatMul_1", [pr, v], T=F32, adj_x=False, adj_y=False)
                            ctx = g.node("Transpose", "transpose_3",
                                         [ctx, g.const("transpose_3/perm", np.array([0, 2, 1, 3], np.int32))],
                                         T=F32, Tperm=I32)
                            ctx = g.node("Reshape", "Reshape_3",
                                         [ctx, g.const("Reshape_3/shape", np.array([-1, Hd], np.int32))], T=F32)
                        with g.scope("output"):
                            ao = dense(g, ctx, Hd, Hd, rng, "dense")
                            ao = g.node("AddV2", "add", [ao, x], T=F32)
                            ao = layer_norm(g, ao, Hd, rng, cfg.eps, "LayerNorm")
                    with g.scope("intermediate"):
                        it = dense(g, ao, Hd, cfg.intermediate, rng, "dense", act="gelu")
                    with g.scope("output"):
                        lo = dense(g, it, cfg.intermediate, Hd, rng, "dense")
                        lo = g.node("AddV2", "add", [lo, ao], T=F32)
                        x = layer_norm(g, lo, Hd, rng, cfg.eps, "LayerNorm")
            seq = g.node("Reshape", "Reshape_2", [x, g.const("Reshape_2/shape", np.array([-1, S, Hd], np.int32))],
                         T=F32)
        with g.scope("pooler"):
            first = g.node("StridedSlice", "strided_slice",
                           [seq, g.const("ss/begin", np.array([0, 0, 0], np.int32)),
                            g.const("ss/end", np.array([0, 1, 0], np.int32)),
                            g.const("ss/strides", np.array([1, 1, 1], np.int32))],
                           T=F32, Index=I32, begin_mask=5, end_mask=5, ellipsis_mask=0, new_axis_mask=0,
                           shrink_axis_mask=0)
            first = g.node("Squeeze", "Squeeze", [first], T=F32, squeeze_dims=[1])
            pooled = dense(g, first, Hd, Hd, rng, "dense", act="tanh")
    with g.scope("loss"):
        logits = dense(g, pooled, Hd, cfg.num_labels, rng, "output")
        probs = g.node("Softmax", "Softmax", [logits], T=F32)
    saver = g.add_saver()
    ins = {n: tensor_info(t, T.DT_INT32, [-1, S]) for n, t in
           (("input_ids", ids), ("input_mask", mask), ("segment_ids", seg))}
    outs = {"probabilities": tensor_info(probs, T.DT_FLOAT, [-1, cfg.num_labels]),
            "pooled_output": tensor_info(pooled, T.DT_FLOAT, [-1, Hd])}
    return g, {"serving_default": signature(ins, outs, PREDICT_METHOD)}, saver


def export(export_dir: str, cfg: BertConfig = BASE, seed: int = 0) -> str:
    g, sigs, saver = build_graph(cfg, seed)
    return write_saved_model(export_dir, g.graph, sigs, g.variables, g.var_dtypes, saver)
