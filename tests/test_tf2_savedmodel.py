"""TF2-layout SavedModels (StatefulPartitionedCall + function library, resource
variables keyed by object path): function inlining, saver-graph variable
binding, and serving through the normal RPC path (CPU)."""
import asyncio
import os

import numpy as np
import pytest

from rust_tensorflow_serving2_amd.graph.ir import from_graph_def, restore_keys
from rust_tensorflow_serving2_amd.models import keras_mlp
from rust_tensorflow_serving2_amd.savedmodel import saved_model as sm
from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions


@pytest.fixture(scope="module")
def mlp_path(tmp_path_factory):
    base = tmp_path_factory.mktemp("tf2") / "mlp"
    keras_mlp.export(str(base / "1"))
    return str(base)


def test_inlining_and_restore_keys(mlp_path):
    b = sm.load(os.path.join(mlp_path, "1"))
    g = from_graph_def(b.graph_def)
    assert not any(n.op in ("PartitionedCall", "StatefulPartitionedCall") for n in g.nodes.values())
    assert g.nodes["StatefulPartitionedCall"].op == "IdentityN"
    keys = restore_keys(g)
    assert keys == dict(zip(keras_mlp.VARS, keras_mlp.KEYS))


def test_tf2_predict_matches_numpy(mlp_path):
    s = Servable("mlp", 1, os.path.join(mlp_path, "1"), ServableOptions(device="cpu"))
    x = np.random.default_rng(3).standard_normal((7, 16)).astype(np.float32)
    out = s.run("serving_default", {"x": x}, ["output_0"])["output_0"]
    ref = keras_mlp.reference(x, keras_mlp.weights())
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


def test_tf2_over_grpc(mlp_path):
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions
    srv = ModelServer(ServerOptions(port=0, model_name="mlp", model_base_path=mlp_path,
                                    file_system_poll_wait_seconds=0)).start()
    try:
        async def go():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(srv.port).build()
            x = np.ones((2, 16), np.float32)
            return x, await c.predict_tensors("mlp", {"x": x})
        x, out = asyncio.run(go())
        np.testing.assert_allclose(out["output_0"], keras_mlp.reference(x, keras_mlp.weights()), rtol=1e-5,
                                   atol=1e-6)
    finally:
        srv.stop()


@pytest.mark.gpu
def test_tf2_on_gpu_fused(mlp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    s = Servable("mlp", 1, os.path.join(mlp_path, "1"), ServableOptions(device="cuda:0", max_batch_size=8))
    x = np.random.default_rng(4).standard_normal((5, 16)).astype(np.float32)
    out = s.run("serving_default", {"x": x}, ["output_0"])["output_0"]
    np.testing.assert_allclose(out, keras_mlp.reference(x, keras_mlp.weights()), atol=2e-2)
