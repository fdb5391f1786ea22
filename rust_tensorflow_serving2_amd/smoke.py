"""One tiny end-to-end forward of the flagship serving path on cuda:0.

Synthetic ResNet SavedModel -> loader -> fusion passes -> gfx950 HIP kernels
(implicit-GEMM MFMA convs, pools, classifier head) -> Predict response bytes,
checked against the fp32 CPU reference interpreter.
"""
from __future__ import annotations

import os
import tempfile

import numpy as np


def run_smoke(device: str = "cuda:0") -> dict:
    import torch
    from . import native
    from .models import resnet
    from .ops import hip
    from .server.core import ServingCore
    from .server.manager import ModelManager
    from .server.servable import Servable, ServableOptions

    assert torch.cuda.is_available(), "smoke needs a GPU"
    hip()   # loud failure if the kernels are not built
    tmp = tempfile.mkdtemp(prefix="tfserve_smoke_")
    base = os.path.join(tmp, "resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=17, image_size=64, seed=3)
    opts = ServableOptions(device=device, max_batch_size=4)

    def loader(name, version, path, cfg):
        return Servable(name, version, path, opts)
    mgr = ModelManager(loader, poll_wait_seconds=0)
    from .schema import serving
    cfg = serving.ModelServerConfig()
    cfg.model_config_list.config.add(name="resnet", base_path=base, model_platform="tensorflow")
    errs = mgr.apply_config(cfg)
    assert not errs, errs
    core = ServingCore(mgr)
    x = np.random.default_rng(0).random((2, 64, 64, 3), dtype=np.float32)
    req = native.encode_predict_request(native.spec_tuple("resnet", None, None, "serving_default"), {"input": x})
    resp = core.predict(req)
    _spec, outs, _f, _d = native.decode_predict_request(_as_request(resp))
    probs = outs["probabilities"]
    # fp32 CPU reference of the same SavedModel
    ref = Servable("resnet", 1, os.path.join(base, "1"), ServableOptions(device="cpu"))
    rout = ref.run("serving_default", {"input": x}, ["classes", "probabilities"])
    err = float(np.abs(probs - rout["probabilities"]).max())
    assert probs.shape == (2, 17) and err < 2e-2, err
    mgr.stop()
    result = {"max_abs_err_vs_fp32": err, "classes": outs["classes"].tolist(),
              "ref_classes": rout["classes"].tolist()}
    print("smoke ok", result)
    return result


def _as_request(resp: bytes) -> bytes:
    """Re-wrap PredictResponse outputs as PredictRequest inputs to reuse the decoder."""
    from .schema import serving
    r = serving.PredictResponse.FromString(resp)
    q = serving.PredictRequest()
    for k, v in r.outputs.items():
        q.inputs[k].CopyFrom(v)
    return q.SerializeToString()


if __name__ == "__main__":
    run_smoke()
