"""ResNet-50 v1.5 (random init) end to end on the GPU runtime vs the fp32 CPU
reference interpreter of the same SavedModel (BASELINE config 2 shape)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)


@pytest.fixture(scope="module")
def resnet50(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50"))
    resnet.export(os.path.join(base, "1"), seed=0)
    return os.path.join(base, "1")


def _check_logits_and_classes(g, c):
    """bf16 GPU vs fp32 CPU: logits (recovered as centred log-probabilities)
    within 5 % of their spread, and the same top-1 class wherever the fp32
    top-1 / top-2 margin exceeds 3x the observed logit error."""
    lg = np.log(np.maximum(g["probabilities"], 1e-30)).astype(np.float64)
    lc = np.log(np.maximum(c["probabilities"], 1e-30)).astype(np.float64)
    lg -= lg.mean(1, keepdims=True)
    lc -= lc.mean(1, keepdims=True)
    err = np.abs(lg - lc).max(1)
    rel = err / lc.std(1)
    assert rel.max() < 5e-2, rel
    top2 = np.sort(lc, 1)[:, -2:]
    decided = (top2[:, 1] - top2[:, 0]) > 3 * err
    assert decided.any()
    np.testing.assert_array_equal(g["classes"][decided], c["classes"][decided])
    return rel.max()


def test_resnet50_gpu_matches_cpu(resnet50):
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    gpu = Servable("resnet", 1, resnet50, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("resnet", 1, resnet50, ServableOptions(device="cpu"))
    x = np.random.default_rng(1).random((5, 224, 224, 3), dtype=np.float32)
    g = gpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    c = cpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    assert g["probabilities"].shape == (5, 1001)
    np.testing.assert_allclose(g["probabilities"].sum(1), 1.0, atol=1e-4)
    err = np.abs(g["probabilities"] - c["probabilities"]).max()
    assert err < 5e-3, err
    _check_logits_and_classes(g, c)
    # run again (HIP-graph replay path, different batch inside the same bucket)
    g2 = gpu.run("serving_default", {"input": x[:3]}, ["classes", "probabilities"])
    # bucket 4 vs bucket 8 may pick different tile/split-K configs -> fp32 summation order differs
    np.testing.assert_allclose(g2["probabilities"], g["probabilities"][:3], atol=2e-4)
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram()
    # 53 convs: 4 stage-entry (expand conv + projection shortcut) pairs run as
    # one K-concatenated dual-source GEMM each
    # the stem conv runs inside the fused stem + max-pool kernel
    assert hist.get("_FusedDualConv") == 4 and "Conv2D" not in hist
    assert hist.get("_StemPool") == 1 and "_MaxPool" not in hist
    assert hist.get("_FusedConv2D") + 2 * hist["_FusedDualConv"] + hist["_StemPool"] == 53


@pytest.fixture(scope="module")
def resnet50_v2(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("r50v2"))
    resnet.export(os.path.join(base, "1"), version="v2", seed=2)
    return os.path.join(base, "1")


def test_resnet50_v2_gpu_fully_fused_matches_cpu(resnet50_v2):
    """ResNet-50 v2 -- the model the reference serves (serving/fetch.sh:7,
    resnet_v2_fp32_savedmodel_NHWC): pre-activation BN+ReLU ride on the
    producing conv / pool epilogues, so the GPU program has no BN, ReLU or Mul
    node left; logits and classes match the fp32 CPU interpreter."""
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    gpu = Servable("resnet", 1, resnet50_v2, ServableOptions(device="cuda:0", max_batch_size=8))
    cpu = Servable("resnet", 1, resnet50_v2, ServableOptions(device="cpu"))
    x = np.random.default_rng(3).random((6, 224, 224, 3), dtype=np.float32)
    g = gpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    c = cpu.run("serving_default", {"input": x}, ["classes", "probabilities"])
    np.testing.assert_allclose(g["probabilities"].sum(1), 1.0, atol=1e-4)
    _check_logits_and_classes(g, c)
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram()
    for op in ("FusedBatchNormV3", "Relu", "Mul", "Conv2D", "AddV2"):
        assert op not in hist, hist
    assert hist.get("_StemPool") == 1 and "_MaxPool" not in hist
    assert hist.get("_FusedConv2D") + 2 * hist.get("_FusedDualConv", 0) + hist["_StemPool"] == 53


def test_smoke():
    from rust_tensorflow_serving2_amd.smoke import run_smoke
    run_smoke()
