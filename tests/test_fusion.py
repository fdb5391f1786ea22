"""Fusion passes on CPU: fused graph (fp32 reference of the fused ops, same
folded parameters the HIP kernels use) == unfused reference interpreter, and
the expected patterns were actually matched."""
import os

import numpy as np
import pytest

from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions


@pytest.fixture(scope="module")
def tiny_bert(models_dir):
    from rust_tensorflow_serving2_amd.models import bert
    cfg = bert.BertConfig(vocab_size=100, hidden=64, layers=2, heads=2, intermediate=128, max_position=64, seq_len=32)
    path = os.path.join(str(models_dir), "tiny_bert", "1")
    bert.export(path, cfg, seed=3)
    return path


def _pair(path):
    return (Servable("m", 1, path, ServableOptions(device="cpu")),
            Servable("m", 1, path, ServableOptions(device="cpu", fuse=True)))


def test_resnet_fusion_exact(tiny_resnet_path):
    ref, fused = _pair(os.path.join(tiny_resnet_path, "1"))
    x = np.random.default_rng(0).random((3, 32, 32, 3), dtype=np.float32)
    a = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    b = fused.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(a["probabilities"], b["probabilities"], atol=1e-5)
    np.testing.assert_array_equal(a["classes"], b["classes"])
    hist = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program.op_histogram()
    assert hist["_FusedConv2D"] == 17 and "Conv2D" not in hist and "FusedBatchNormV3" not in hist
    # GlobalAvgPool -> dense -> softmax/argmax is one classifier-head op
    assert hist["_ClassifierHead"] == 1 and hist["_MaxPool"] == 1
    assert "_SoftmaxArgMax" not in hist and "_GlobalAvgPool" not in hist and "_FusedMatMul" not in hist


@pytest.fixture(scope="module")
def tiny_resnet_v2_path(models_dir):
    from rust_tensorflow_serving2_amd.models import resnet
    base = os.path.join(str(models_dir), "tiny_resnet_v2")
    resnet.export(os.path.join(base, "1"), version="v2", blocks=(2, 2, 1, 1), width=8, num_classes=11,
                  image_size=32, seed=4)
    return base


def test_resnet_v2_preactivation_fully_fused(tiny_resnet_v2_path):
    """ResNet v2 (the reference's model, serving/fetch.sh:7): every
    pre-activation BN + ReLU rides on the producing conv / dual conv / pool as
    its post-activation output, the residual scale folds into conv3's weights:
    no FusedBatchNorm, Relu or Mul node is left."""
    ref, fused = _pair(os.path.join(tiny_resnet_v2_path, "1"))
    x = np.random.default_rng(1).random((3, 32, 32, 3), dtype=np.float32)
    a = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    b = fused.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(a["probabilities"], b["probabilities"], atol=1e-5)
    np.testing.assert_array_equal(a["classes"], b["classes"])
    hist = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program.op_histogram()
    for op in ("FusedBatchNormV3", "Relu", "Mul", "Conv2D", "AddV2"):
        assert op not in hist, hist
    assert hist["_MaxPool"] == 1 and hist["_ClassifierHead"] == 1


@pytest.mark.parametrize("version", ["v1.5", "v2"])
def test_resnet_stem_conv_and_pool_become_one_op(models_dir, version):
    """The 7x7/2 RGB stem conv and the 3x3/2 max pool after it fuse into
    _StemPool (one kernel on the GPU); on the CPU it is the same composition."""
    from rust_tensorflow_serving2_amd.models import resnet
    path = os.path.join(str(models_dir), f"stem_{version}", "1")
    resnet.export(path, version=version, blocks=(1, 1, 1, 1), width=16, num_classes=7, image_size=40, seed=3)
    ref, fused = _pair(path)
    x = np.random.default_rng(2).random((2, 40, 40, 3), dtype=np.float32)
    a = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    b = fused.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(a["probabilities"], b["probabilities"], atol=1e-5)
    np.testing.assert_array_equal(a["classes"], b["classes"])
    prog = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program
    hist = prog.op_histogram()
    assert hist["_StemPool"] == 1 and "_MaxPool" not in hist, hist
    # the replicated-weights packer (graph/placement.py) must see the stem conv
    # nested inside the fused op, or a follower replica would keep its own copy
    from rust_tensorflow_serving2_amd.graph.placement import weight_refs
    stem = next(n.attrs["_impl"] for _f, n, _i, _o in prog.steps if n.op == "_StemPool")
    held = {id(ref[0]) for ref, _t in weight_refs(prog)}
    assert id(stem.conv) in held


def test_bert_fusion_exact(tiny_bert):
    ref, fused = _pair(tiny_bert)
    rng = np.random.default_rng(0)
    ids = rng.integers(0, 100, (3, 32)).astype(np.int32)
    mask = np.ones((3, 32), np.int32)
    mask[1, 20:] = 0
    seg = np.zeros((3, 32), np.int32)
    seg[:, 16:] = 1
    feeds = {"input_ids": ids, "input_mask": mask, "segment_ids": seg}
    outs = ["pooled_output", "probabilities"]
    a, b = ref.run("serving_default", feeds, outs), fused.run("serving_default", feeds, outs)
    for k in outs:
        np.testing.assert_allclose(a[k], b[k], atol=1e-5)
    hist = fused.runner("serving_default", sorted(feeds), outs).program.op_histogram()
    assert hist["_LayerNorm"] == 4 and hist["_Attention"] == 2 and hist["_FusedQKV"] == 2
    # embedding gathers + adds + LN -> one op; the [B,S,S] mask adder chain -> one [B,1,1,S] op
    assert hist["_EmbeddingLN"] == 1 and hist["_KeyMaskAdder"] == 1
    assert "GatherV2" not in hist and "ExpandDims" not in hist and "Cast" not in hist
    # (the 2-label classifier + softmax is one _DenseSoftmax op)
    assert hist["_FusedMatMul"] == 7 and hist["_DenseSoftmax"] == 1 and "Softmax" not in hist
    assert "MatMul" not in hist and "BatchMatMulV2" not in hist
    assert "Rsqrt" not in hist and "Pow" not in hist and "Tanh" not in hist


def test_bert_fused_embedding_rejects_out_of_range_ids_on_cpu(tiny_bert):
    """The fused embedding keeps GatherV2's CPU contract: an id outside the
    vocabulary is an error, as in the unfused graph."""
    from rust_tensorflow_serving2_amd.server.errors import ServingError
    _ref, fused = _pair(tiny_bert)
    ids = np.full((1, 32), 5, np.int32)
    ids[0, 3] = 100                                 # vocab_size == 100
    feeds = {"input_ids": ids, "input_mask": np.ones((1, 32), np.int32), "segment_ids": np.zeros((1, 32), np.int32)}
    with pytest.raises(ServingError, match="out of range"):
        fused.run("serving_default", feeds, ["pooled_output"])


def test_gelu_erf_form_matches():
    """Keras-style erf GELU subgraph is recognised too."""
    import torch
    from rust_tensorflow_serving2_amd.graph.builder import DType, GraphBuilder
    from rust_tensorflow_serving2_amd.graph.compiler import compile_program
    from rust_tensorflow_serving2_amd.graph.fused import default_passes
    from rust_tensorflow_serving2_amd.graph.ir import from_graph_def
    from rust_tensorflow_serving2_amd.utils import tensors as T
    f32 = DType(T.DT_FLOAT)
    g = GraphBuilder()
    x = g.placeholder("x", T.DT_FLOAT, [-1, 16])
    w = g.const("w", np.random.default_rng(0).standard_normal((16, 24)).astype(np.float32))
    y = g.node("MatMul", "mm", [x, w], T=f32)
    half = g.node("Mul", "half", [y, g.const("c05", np.float32(0.5))], T=f32)
    d = g.node("RealDiv", "div", [y, g.const("sq2", np.float32(np.sqrt(2)))], T=f32)
    e = g.node("Erf", "erf", [d], T=f32)
    a = g.node("AddV2", "add", [g.const("one", np.float32(1.0)), e], T=f32)
    out = g.node("Mul", "gelu", [half, a], T=f32)
    xs = torch.randn(5, 16)
    p0 = compile_program(from_graph_def(g.graph), ["x:0"], [out + ":0"])
    p1 = compile_program(from_graph_def(g.graph), ["x:0"], [out + ":0"], passes=default_passes())
    assert p1.op_histogram() == {"_FusedMatMul": 1}
    torch.testing.assert_close(p0.run([xs])[0], p1.run([xs])[0], atol=1e-5, rtol=1e-5)


def test_tuned_cache_roundtrip(tmp_path, monkeypatch):
    """A committed tile-pick table is installed only when its schema matches
    (stale config ids are never launched)."""
    import json
    from rust_tensorflow_serving2_amd import ops
    monkeypatch.setattr(ops, "_REMOTE", {})
    p = tmp_path / "t.json"
    key = ("mm", 32, 768, 768, False, True, "tanh")
    p.write_text(json.dumps({"schema": ops._table_schema(), "arch": "gfx950", "cus": 256,
                             "picks": {repr(key): [42, 1]}}))
    assert ops.load_tuned_cache(str(p)) == 1 and ops._REMOTE[repr(key)] == (42, 1)
    monkeypatch.setattr(ops, "_REMOTE", {})
    p.write_text(json.dumps({"schema": "stale", "picks": {repr(key): [42, 1]}}))
    assert ops.load_tuned_cache(str(p)) == 0 and not ops._REMOTE


def test_committed_tuned_table_matches_config_schema():
    """The shipped MI355X table (ops/tuned_mi355x.json) must carry the schema
    of the current config tables: a stale one is silently ignored at start-up
    and every server re-tunes its kernels (round 6 found the table stale after
    the ping-pong config ids went in)."""
    import json
    from rust_tensorflow_serving2_amd import ops
    with open(os.path.join(os.path.dirname(ops.__file__), "tuned_mi355x.json")) as f:
        doc = json.load(f)
    assert doc["schema"] == ops._table_schema()
    assert doc["arch"] == "gfx950" and doc["cus"] == 256 and len(doc["picks"]) > 100
    assert all(int(v[0]) in ops.TILES for v in doc["picks"].values())


def test_conv_chain_pass_pairs_expand_with_next_reduce(models_dir, monkeypatch):
    """ResNet-50 stage-1/2 widths: every 1x1 expand whose output feeds the next
    block's 1x1 reduce becomes one _ChainConv with outputs [expand, reduce]
    (7 pairs on CPU; on the GPU the two projecting blocks' expands are dual
    convs first, leaving 5); the fused program still equals the unfused
    interpreter."""
    from rust_tensorflow_serving2_amd.models import resnet
    monkeypatch.setenv("TFSERVE_CONV_CHAIN", "force")     # the pass is GPU-only by default
    monkeypatch.setenv("TFSERVE_CONV_CHAIN_SHAPES", "all")
    path = os.path.join(str(models_dir), "chain_resnet", "1")
    resnet.export(path, blocks=(3, 4, 1, 1), width=64, num_classes=10, image_size=32, seed=5)
    ref, fused = _pair(path)
    x = np.random.default_rng(2).random((2, 32, 32, 3), dtype=np.float32)
    a = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    b = fused.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(a["probabilities"], b["probabilities"], atol=1e-5)
    np.testing.assert_array_equal(a["classes"], b["classes"])
    hist = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program.op_histogram()
    assert hist["_ChainConv"] == 7 - hist.get("_FusedDualConv", 0), hist
    convs = 3 * 9 + 4                                     # 9 blocks x 3 + 4 projections (the stem is in _StemPool)
    assert hist["_StemPool"] == 1
    assert hist["_FusedConv2D"] + 2 * hist["_ChainConv"] + 2 * hist.get("_FusedDualConv", 0) == convs, hist


def test_activation_release_plan(tiny_resnet_path):
    """The program drops each value after its last reader (compile-time
    liveness): results are unchanged and far fewer values are alive at once."""
    from rust_tensorflow_serving2_amd.graph.compiler import plan_release
    fused = Servable("m", 1, os.path.join(tiny_resnet_path, "1"), ServableOptions(device="cpu", fuse=True))
    prog = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program
    plan = prog.activation_plan()
    assert plan["peak_live_values"] <= 4 < plan["values"], plan
    # no fetched, fed or constant slot is ever released
    keep = set(prog.fetch_slots) | set(prog.feed_slots) | {s for s, _v in prog.const_slots}
    assert not keep & {s for dead in prog.free_after for s in dead}
    x = np.random.default_rng(3).random((2, 32, 32, 3), dtype=np.float32)
    import torch
    a = [t.clone() if hasattr(t, "clone") else t for t in prog.run([torch.from_numpy(x)])]
    prog.free_after = [[] for _ in prog.steps]            # keep everything: the old behaviour
    b = prog.run([torch.from_numpy(x)])
    for u, v in zip(a, b):
        np.testing.assert_array_equal(np.asarray(u), np.asarray(v))
    assert plan_release([], 0, [], [], []) == []


def test_capture_holds_off_gc_across_nested_and_threaded_captures():
    """Graph captures run with Python's GC off (ops._no_gc: a collection there
    can run a dead server's CUDAGraph destructor on the capturing thread);
    counted, so overlapping captures on two threads re-enable it only when
    the last one ends, and a GC the caller had disabled stays disabled."""
    import gc
    import threading
    from rust_tensorflow_serving2_amd import ops
    assert gc.isenabled()
    inside, release = threading.Event(), threading.Event()

    def other():
        with ops._no_gc():
            inside.set()
            release.wait(10)

    t = threading.Thread(target=other)
    t.start()
    assert inside.wait(10)
    with ops._no_gc():
        assert not gc.isenabled()
    assert not gc.isenabled()           # the other thread's capture still runs
    release.set()
    t.join()
    assert gc.isenabled()
    gc.disable()
    try:
        with ops._no_gc():
            pass
        assert not gc.isenabled()
    finally:
        gc.enable()


def test_defer_layernorm_pass_rewires_and_matches_unfused():
    """defer_layernorm on a hand-built encoder slice (producer GEMM -> LN ->
    {A of a GELU GEMM, residual of another GEMM}): the LN node goes, the
    readers take the raw sum plus the producer's row partials, and the folded
    math (DeferredLNMatMul._reference, the kernel's algebra in fp32) matches
    the materialised LayerNorm.  The pass itself only runs for GPU programs;
    it is driven here with CPU-built ops and a cuda device tag."""
    import torch
    import torch.nn.functional as F
    from rust_tensorflow_serving2_amd.graph import fused as FU
    from rust_tensorflow_serving2_amd.graph.ir import Graph, Node
    from rust_tensorflow_serving2_amd.graph.patterns import LayerNormOp

    torch.manual_seed(0)
    cpu = torch.device("cpu")
    C, F4 = 64, 128
    w0, w1, w2 = torch.randn(C, C) / 8, torch.randn(C, F4) / 8, torch.randn(F4, C) / 11
    b0, b1, b2 = torch.randn(C) / 10, torch.randn(F4) / 10, torch.randn(C) / 10
    gam, bet = 1 + torch.randn(C) / 10, torch.randn(C) / 10
    mm0 = FU.FusedMatMul(w0, b0, "none", False, cpu, True, "p")
    mm1 = FU.FusedMatMul(w1, b1, "gelu_tanh", False, cpu, True, "a")
    mm2 = FU.FusedMatMul(w2, b2, "none", False, cpu, True, "r")
    ln = LayerNormOp(gam, bet, 1e-6, cpu, True)
    g = Graph()
    g.add(Node(name="x", op="Placeholder"))
    g.add(Node(name="p", op="_FusedMatMul", inputs=[("x", 0), ("x", 0)], attrs={"_impl": mm0}))
    g.add(Node(name="ln", op="_LayerNorm", inputs=[("p", 0)], attrs={"_impl": ln}))
    g.add(Node(name="a", op="_FusedMatMul", inputs=[("ln", 0)], attrs={"_impl": mm1}))
    g.add(Node(name="r", op="_FusedMatMul", inputs=[("a", 0), ("ln", 0)], attrs={"_impl": mm2}))
    order = ["x", "p", "ln", "a", "r"]
    x = torch.randn(16, C).to(torch.bfloat16)

    # unfused: LN materialised (bf16 like the GPU program)
    bf = torch.bfloat16
    zp = (x.float() @ w0.to(bf).float() + b0 + x.float()).to(bf)
    h = F.layer_norm(zp.float(), (C,), gam, bet, 1e-6)
    a_ref = F.gelu(h.to(bf).float() @ w1 + b1, approximate="tanh")
    r_ref = a_ref.to(bf).float() @ w2 + b2 + h

    os.environ["TFSERVE_DEFER_LN"] = "1"
    try:
        FU.defer_layernorm(g, order, set(), [("r", 0)], torch.device("cuda"), None)
    finally:
        del os.environ["TFSERVE_DEFER_LN"]
    FU.release_weight_sources(g, order, set(), [("r", 0)], torch.device("cuda"), None)
    assert "ln" not in g.nodes
    assert g.nodes["a"].inputs == [("p", 0), ("p", 1)]
    assert g.nodes["r"].inputs == [("a", 0), ("p", 0), ("p", 1)]
    P, A, R = (g.nodes[k].attrs["_impl"] for k in "par")
    assert P.emit and A.a_ln is not None and A.a_pos == 1 and R.r_ln is not None and R.r_pos == 2
    assert R.has_res and not A.has_res and P.has_res
    assert all(m._w_src is None for m in (P, A, R))

    zz, st = P(None, g.nodes["p"], [x, x])
    assert st.shape == (16, 1, 2)
    assert torch.allclose(zz.float(), zp.float(), atol=2e-2, rtol=1e-2)
    assert torch.allclose(st[:, :, 0].sum(1), zz.float().sum(1), rtol=1e-5, atol=1e-4)
    aa = A(None, g.nodes["a"], [zz, st])[0]
    rr = R(None, g.nodes["r"], [aa, zz, st])[0]
    assert (aa.float() - a_ref).abs().max() < 5e-2
    assert (rr.float() - r_ref).abs().max() < 8e-2


def test_defer_layernorm_leaves_other_readers_alone():
    """A LayerNorm read by anything but GEMM inputs (here a fetch) stays."""
    import torch
    from rust_tensorflow_serving2_amd.graph import fused as FU
    from rust_tensorflow_serving2_amd.graph.ir import Graph, Node
    from rust_tensorflow_serving2_amd.graph.patterns import LayerNormOp

    cpu = torch.device("cpu")
    mm0 = FU.FusedMatMul(torch.randn(64, 64), None, "none", False, cpu, True, "p")
    mm1 = FU.FusedMatMul(torch.randn(64, 64), None, "none", False, cpu, True, "a")
    g = Graph()
    g.add(Node(name="x", op="Placeholder"))
    g.add(Node(name="p", op="_FusedMatMul", inputs=[("x", 0)], attrs={"_impl": mm0}))
    g.add(Node(name="ln", op="_LayerNorm", inputs=[("p", 0)],
               attrs={"_impl": LayerNormOp(torch.ones(64), torch.zeros(64), 1e-6, cpu, True)}))
    g.add(Node(name="a", op="_FusedMatMul", inputs=[("ln", 0)], attrs={"_impl": mm1}))
    order = ["x", "p", "ln", "a"]
    FU.defer_layernorm(g, order, set(), [("a", 0)], torch.device("cuda"), None)    # opt-in: off by default
    assert "ln" in g.nodes
    os.environ["TFSERVE_DEFER_LN"] = "1"
    try:
        FU.defer_layernorm(g, order, set(), [("a", 0), ("ln", 0)], torch.device("cuda"), None)
    finally:
        del os.environ["TFSERVE_DEFER_LN"]
    assert "ln" in g.nodes and g.nodes["a"].inputs == [("ln", 0)]
    FU.defer_layernorm(g, order, set(), [("a", 0)], torch.device("cpu"), None)   # CPU programs: never
    assert "ln" in g.nodes


def test_tile_candidates_respect_kernel_limits():
    """ops.candidates: the tuner is only offered tiles the launchers accept --
    no big-tile (bgemm) build for the padded RGBA stem or the deferred
    LayerNorm, only 4-aligned chunk-lane cgemm tiles for the deferred
    LayerNorm, and 144- / 96-wide tiles only where they divide N; the retired
    ids 124..137 are gone."""
    from rust_tensorflow_serving2_amd import ops
    qkv = ops.candidates(4096, 2304, 768, True, True)
    assert (73, 1) in qkv and (72, 1) in qkv and (140, 1) in qkv and (141, 1) in qkv
    assert all(c not in range(124, 138) for c, _s in qkv)
    assert all(c != 73 for c, _s in ops.candidates(4096, 3072, 768, True, True))    # 3072 % 144 != 0
    stem = ops.candidates(32 * 112 * 112, 64, 128, False, True, stem=True)
    assert stem and all(c not in ops.BGEMM for c, _s in stem)
    ln = ops.candidates(4096, 768, 3072, True, True, no_split=True, ln=True)
    assert ln and all(s == 1 and c in ops.CGEMM and c not in ops.BGEMM and ops.TILES[c][1] % 32 == 0
                      for c, s in ln)