"""The flow kernel's step table (graph/flow.py) checked on the CPU: a Python
interpreter of the table -- the same pointer decoding, operand modes (dense /
im2col with padding and stride / dual [h | strided x]), dependency fields and
split-K bookkeeping kernels/flow.hip reads -- must reproduce an fp32 torch
computation of the chain, and the fusion pass must leave the served model's
results unchanged when the block runs its member ops one by one."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from rust_tensorflow_serving2_amd.graph import flow
from rust_tensorflow_serving2_amd.graph.fused import ChainConv, FusedConv, FusedDualConv

CPU = torch.device("cpu")


def _conv(cin, cout, k, s, act, seed, padding="SAME"):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(k, k, cin, cout, generator=g) / (k * k * cin) ** 0.5
    b = torch.randn(cout, generator=g) * 0.1
    return FusedConv(w, b, (s, s), padding, None, act, CPU, True, f"c{seed}")


def _ref_conv(impl: FusedConv, x, res=None):
    """fp32 NHWC conv of the impl's bf16 weights (what the kernels multiply)."""
    k = impl.kh * impl.kw * impl.cin
    w = impl.w[:, :k].float().reshape(impl.cout, impl.kh, impl.kw, impl.cin).permute(0, 3, 1, 2)
    pt, pb, pl, pr = impl.pads_for(x.shape[1], x.shape[2])
    y = F.conv2d(F.pad(x.permute(0, 3, 1, 2), [pl, pr, pt, pb]), w, stride=(impl.sh, impl.sw))
    y = y.permute(0, 2, 3, 1) + impl.b
    if res is not None:
        y = y + res
    return torch.relu(y) if impl.act == "relu" else y


def _interpret(tab, x, weights):
    """Run the table the way flow_kernel does (whole steps, fp32)."""
    t = tab["table"]
    nsteps = tab["nsteps"]
    arena = torch.zeros(tab["arena"] // 4 + 1, dtype=torch.float32)        # fp32 shadow, byte offsets / 2 -> elems
    store = {}                                                              # (kind, off) -> fp32 tensor

    def get(ref, shape):
        kind, off = ref >> flow.REF_SHIFT, ref & ((1 << flow.REF_SHIFT) - 1)
        if kind == flow.K_ABS:
            return weights[off]
        if kind == flow.K_ENTRY:
            assert off == 0
            return x.reshape(shape)
        return store[(kind, off)].reshape(shape)

    starts = t[:flow.MAX_STEPS]
    done = set()
    rows_seen = set()
    last_task = 0
    for i in range(nsteps):
        f = t[flow.MAX_STEPS + i * flow.STEP_INTS:flow.MAX_STEPS + (i + 1) * flow.STEP_INTS]
        refs = f[:16].view(np.int64).tolist()
        (M, N, K, K1, lda, ldb, H, W, C, Ho, Wo, KH, KW, SH, SW, PT, PL, mode, act, ntm, ntn, splits, ktps, ntasks,
         d0, d1, d2, ctr, a_bytes, a2_bytes, b_bytes, rctr) = f[16:].tolist()
        assert starts[i] == last_task and ntasks == ntm * ntn * splits and ntm == -(-M // 32) and ntn == -(-N // 64)
        assert ktps * splits >= K // 64 > ktps * (splits - 1) and K % 64 == 0
        assert (refs[6] != flow.NULL_REF) == (splits > 1) and (ctr >= flow.CTRL_HEAD) == (splits > 1)
        assert rctr % flow.ROW_STRIDE == 0 and rctr + ntm * flow.ROW_STRIDE <= tab["ctrl_ints"]
        assert rctr not in rows_seen and (splits == 1 or ctr + ntm * ntn <= min(rows_seen | {rctr}))
        rows_seen.add(rctr)
        last_task += ntasks
        for d in (d0, d1, d2):
            assert d < i and (d < 0 or d in done)
        a_ref, a2_ref, w_ref, b_ref, r_ref, o_ref = refs[:6]
        wt = get(w_ref, None)
        assert b_bytes == wt.numel() * 2 and wt.shape[1] == ldb
        wk = wt[:N, :K].float()
        if mode == flow.MODE_DENSE:
            A = get(a_ref, (M, lda))[:, :K]
            assert a_bytes == M * lda * 2
        elif mode == flow.MODE_DUAL:
            h = get(a_ref, (M, K1))
            xs = get(a2_ref, (-1, H, W, C))
            assert a2_bytes == xs.numel() * 2
            A = torch.cat([h, xs[:, ::SH, ::SW, :].reshape(M, C)], dim=1)
        else:
            xi = get(a_ref, (-1, H, W, C))
            assert a_bytes == xi.numel() * 2
            nb = xi.shape[0]
            pb = max(0, (Ho - 1) * SH + KH - H - PT)
            pr = max(0, (Wo - 1) * SW + KW - W - PL)
            xp = F.pad(xi.permute(0, 3, 1, 2), [PL, pr, PT, pb])
            cols = F.unfold(xp, (KH, KW), stride=(SH, SW))                   # [n, C*KH*KW, L], (c, kh, kw)
            cols = cols.reshape(nb, C, KH * KW, -1).permute(0, 3, 2, 1)      # -> k = tap * C + c
            A = cols.reshape(M, K)
        y = A @ wk.t()
        if b_ref != flow.NULL_REF:
            y = y + get(b_ref, None)
        if r_ref != flow.NULL_REF:
            y = y + get(r_ref, (M, N))
        y = torch.relu(y) if act == 1 else y
        kind, off = o_ref >> flow.REF_SHIFT, o_ref & ((1 << flow.REF_SHIFT) - 1)
        assert kind in (flow.K_ARENA, flow.K_OUT)
        if kind == flow.K_ARENA:
            assert off % 256 == 0 and off + M * N * 2 <= tab["arena"]
        store[(kind, off)] = y
        done.add(i)
    assert last_task == tab["ntasks"] and all(s == np.iinfo(np.int32).max for s in starts[nsteps:])
    del arena
    return store[(flow.K_OUT, 0)]


def _chain(width=64):
    """Two bottlenecks: a projecting stride-2 one (3x3 stride 2, v1.5) then an
    identity one whose expand is chained with a following reduce."""
    w = width
    r1, c1 = _conv(w, w, 1, 1, "relu", 1), _conv(w, w, 3, 2, "relu", 2)
    e1, p1 = _conv(w, 4 * w, 1, 1, "relu", 3), _conv(w, 4 * w, 1, 2, "none", 4)
    dual = FusedDualConv(e1, p1, "relu", CPU, True, "d")
    r2, c2, e2 = _conv(4 * w, w, 1, 1, "relu", 5), _conv(w, w, 3, 1, "relu", 6), _conv(w, 4 * w, 1, 1, "relu", 7)
    r3 = _conv(4 * w, 2 * w, 1, 1, "relu", 8)
    subs = [(r1, None, [0], [1]), (c1, None, [1], [2]), (dual, None, [2, 0], [3]),
            (r2, None, [3], [4]), (c2, None, [4], [5]), (ChainConv(e2, r3), None, [5, 3], [6, 7])]
    block = flow.FlowBlock(subs, 7, "t")

    def ref(x):
        a = _ref_conv(r1, x)
        b = _ref_conv(c1, a)
        d = torch.relu(F.conv2d(b.permute(0, 3, 1, 2), _w(e1)).permute(0, 2, 3, 1) + e1.b +
                       F.conv2d(x.permute(0, 3, 1, 2), _w(p1), stride=2).permute(0, 2, 3, 1) + p1.b)
        f = _ref_conv(r2, d)
        g = _ref_conv(c2, f)
        h = _ref_conv(e2, g, res=d)
        return _ref_conv(r3, h)
    return block, ref, [r1, c1, dual, r2, c2, e2, r3]


def _w(impl):
    k = impl.kh * impl.kw * impl.cin
    return impl.w[:, :k].float().reshape(impl.cout, impl.kh, impl.kw, impl.cin).permute(0, 3, 1, 2)


@pytest.mark.parametrize("batch,target", [(1, 256), (2, 256), (3, 64)])
def test_flow_table_interpreter_matches_fp32(batch, target, monkeypatch):
    monkeypatch.setenv("TFSERVE_FLOW_MAX_SPLITS", "16")
    block, ref, impls = _chain()
    x = torch.rand(batch, 12, 12, 64)
    tab = block.build_table(tuple(x.shape), target_tasks=target)
    assert tab["nsteps"] == 7 and tab["ctrl_ints"] >= flow.CTRL_HEAD + 7 * flow.ROW_STRIDE
    assert any(s["splits"] > 1 for s in tab["steps"])          # K-sliced layers exercised
    weights = {}
    for impl in impls:
        weights[impl.w.data_ptr()] = impl.w
        weights[impl.b.data_ptr()] = impl.b
    y = _interpret(tab, x, weights)
    want = ref(x)
    assert y.shape == (batch * 6 * 6, 128)
    torch.testing.assert_close(y.reshape(want.shape), want, rtol=1e-4, atol=1e-4)


def test_pick_splits(monkeypatch):
    assert flow.pick_splits(16, 32, 256) == (1, 32)          # default: no K-slices (measured fastest)
    monkeypatch.setenv("TFSERVE_FLOW_MAX_SPLITS", "16")
    assert flow.pick_splits(300, 64, 256) == (1, 64)
    assert flow.pick_splits(16, 32, 256) == (16, 2)
    assert flow.pick_splits(16, 3, 256) == (1, 3)
    s, per = flow.pick_splits(2, 72, 256)
    assert s * per >= 72 and per >= 2 and s <= 16


def test_flow_pass_on_cpu_runs_members(models_dir, monkeypatch):
    """TFSERVE_FLOW=force on the CPU: the bottleneck stack becomes one
    _FlowBlock that runs its member ops (fp32 references) one by one; results
    equal the unfused interpreter."""
    from rust_tensorflow_serving2_amd.models import resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    monkeypatch.setenv("TFSERVE_FLOW", "force")
    monkeypatch.setenv("TFSERVE_CONV_CHAIN", "force")
    path = os.path.join(str(models_dir), "flow_resnet", "1")
    resnet.export(path, blocks=(2, 2, 1, 1), width=64, num_classes=10, image_size=32, seed=5)
    ref = Servable("m", 1, path, ServableOptions(device="cpu"))
    fused = Servable("m", 1, path, ServableOptions(device="cpu", fuse=True))
    x = np.random.default_rng(2).random((2, 32, 32, 3), dtype=np.float32)
    a = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    b = fused.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(a["probabilities"], b["probabilities"], atol=1e-5)
    prog = fused.runner("serving_default", ["input"], ["classes", "probabilities"]).program
    hist = prog.op_histogram()
    assert hist["_FlowBlock"] == 1 and "_FusedConv2D" not in hist and "_ChainConv" not in hist, hist
    flat = prog.op_histogram(flat=True)
    assert flat["_FusedConv2D"] + 2 * flat.get("_ChainConv", 0) == 3 * 6 + 4, flat
