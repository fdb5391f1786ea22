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
    # run again (HIP-graph replay path, different batch inside the same bucket)
    g2 = gpu.run("serving_default", {"input": x[:3]}, ["classes", "probabilities"])
    # bucket 4 vs bucket 8 may pick different tile/split-K configs -> fp32 summation order differs
    np.testing.assert_allclose(g2["probabilities"], g["probabilities"][:3], atol=2e-4)
    runner = next(iter(gpu._runners.values()))
    hist = runner.program.op_histogram()
    # 53 convs: 4 stage-entry (expand conv + projection shortcut) pairs run as
    # one K-concatenated dual-source GEMM each
    assert hist.get("_FusedDualConv") == 4 and "Conv2D" not in hist
    assert hist.get("_FusedConv2D") + 2 * hist["_FusedDualConv"] == 53


def test_smoke():
    from rust_tensorflow_serving2_amd.smoke import run_smoke
    run_smoke()
