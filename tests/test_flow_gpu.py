"""Persistent dataflow conv chain (kernels/flow.hip, graph/flow.py) on the
GPU: the ResNet-50 bottleneck stack as ONE launch vs the per-layer kernels it
replaces (same bf16 rounding points, different fp32 summation order), the
control words it leaves behind, run-to-run determinism, and the served model
end to end (HIP-graph replays of the flow launch) vs the fp32 CPU reference."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def r50_path(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50flow"))
    resnet.export(os.path.join(base, "1"), seed=0)
    return os.path.join(base, "1")


@pytest.fixture(scope="module")
def r50_gpu(r50_path):
    """The flow pass is opt-in (TFSERVE_FLOW=1); K-slices on, so the in-kernel
    split-K path is exercised too."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    old = {k: os.environ.get(k) for k in ("TFSERVE_FLOW", "TFSERVE_FLOW_MAX_SPLITS")}
    os.environ.update(TFSERVE_FLOW="1", TFSERVE_FLOW_MAX_SPLITS="16")
    try:
        s = Servable("resnet", 1, r50_path, ServableOptions(device="cuda:0", max_batch_size=4))
        s.runner("serving_default", ["input"], ["classes", "probabilities"])
        yield s
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _program(servable):
    return servable.runner("serving_default", ["input"], ["classes", "probabilities"]).program


def _blocks(prog):
    return [n.attrs["_impl"] for _f, n, _i, _o in prog.steps if n.op == "_FlowBlock"]


def test_flow_block_covers_the_bottleneck_stack(r50_gpu):
    prog = _program(r50_gpu)
    (blk,) = _blocks(prog)
    hist = prog.op_histogram()
    assert hist == {"_StemPool": 1, "_FlowBlock": 1, "_ClassifierHead": 1, "Identity": 1} or \
        set(hist) <= {"_StemPool", "_FlowBlock", "_ClassifierHead", "Identity", "Reshape", "Squeeze"}, hist
    # 16 bottlenecks: 3 convs each, the 4 projections merged into dual convs
    assert len(blk.steps((1, 56, 56, 64))) == 48
    flat = prog.op_histogram(flat=True)
    assert flat["_FusedDualConv"] == 4 and flat["_StemPool"] == 1


@pytest.mark.parametrize("batch", [1, 2, 4])
def test_flow_matches_layer_kernels(r50_gpu, batch):
    from rust_tensorflow_serving2_amd.graph import ops as O
    (blk,) = _blocks(_program(r50_gpu))
    gen = torch.Generator(device="cuda").manual_seed(batch)
    x = (torch.rand(batch, 56, 56, 64, device="cuda", generator=gen) * 2).to(torch.bfloat16)
    tab = blk.table_for(x)
    assert tab is not None and tab["ntasks"] > 0
    ctrl = torch.zeros(tab["ctrl_ints"] + 64, dtype=torch.int32, device="cuda")
    y = blk.run_flow(x, ctrl=ctrl)
    y2 = blk.run_flow(x, ctrl=ctrl)
    torch.cuda.synchronize()
    c = ctrl.cpu()
    assert int(c[2]) == 0, "a dependency wait timed out"
    assert int(c[0]) == 0 and int(c[1]) == 0 and int(c[3]) == 2, c[:4].tolist()   # ticket, exit, epoch
    # every row-block counter saw its tiles twice; the split-K arrival counters are back at zero
    for st in tab["steps"]:
        rows = c[st["rctr"]:st["rctr"] + st["ntm"] * 16:16]
        assert (rows == 2 * st["ntn"]).all(), (st["rctr"], rows[:4].tolist(), st["ntn"])
    split_area = c[4:min(st["rctr"] for st in tab["steps"])]
    assert int(split_area.abs().sum()) == 0
    assert torch.equal(y, y2), "flow launch is not deterministic"
    ref = blk.run_sequential(O.Ctx(torch.device("cuda:0")), x)
    assert y.shape == ref.shape == (batch, 7, 7, 2048)
    rel = float((y.float() - ref.float()).norm() / ref.float().norm())
    assert rel < 2e-2, rel
    assert torch.isfinite(y.float()).all()


def test_flow_served_model_matches_cpu(r50_gpu, r50_path):
    """Predict through the HIP-graph replays (buckets 1 / 2 / 4 all run the
    flow launch) vs the fp32 CPU interpreter of the same SavedModel."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    cpu = Servable("resnet", 1, r50_path, ServableOptions(device="cpu"))
    x = np.random.default_rng(7).random((4, 224, 224, 3), dtype=np.float32)
    c = cpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    for n in (1, 3, 4):
        g = r50_gpu.run("serving_default", {"input": x[:n]}, ["classes", "probabilities"])
        g2 = r50_gpu.run("serving_default", {"input": x[:n]}, ["classes", "probabilities"])
        np.testing.assert_array_equal(g["probabilities"], g2["probabilities"])
        np.testing.assert_allclose(g["probabilities"].sum(1), 1.0, atol=1e-4)
        lg = np.log(np.maximum(g["probabilities"], 1e-30)).astype(np.float64)
        lc = np.log(np.maximum(c["probabilities"][:n], 1e-30)).astype(np.float64)
        lg -= lg.mean(1, keepdims=True)
        lc -= lc.mean(1, keepdims=True)
        rel = np.abs(lg - lc).max(1) / lc.std(1)
        assert rel.max() < 5e-2, (n, rel)


def test_flow_disabled_runs_layer_kernels(r50_path, monkeypatch):
    """TFSERVE_FLOW_MAX_BATCH=0: the block runs its member ops one by one."""
    from rust_tensorflow_serving2_amd.graph import flow
    monkeypatch.setenv("TFSERVE_FLOW", "1")
    monkeypatch.setenv("TFSERVE_FLOW_MAX_BATCH", "0")
    assert flow.max_batch() == 0
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    s = Servable("resnet", 1, r50_path, ServableOptions(device="cuda:0", max_batch_size=2))
    (blk,) = _blocks(_program(s))
    x = torch.zeros(1, 56, 56, 64, device="cuda", dtype=torch.bfloat16)
    assert not blk.enabled_for(x)
    g = s.run("serving_default", {"input": np.zeros((1, 224, 224, 3), np.float32)}, ["classes"])
    assert g["classes"].shape == (1,)
