"""BASELINE config 5 at test scale: a ResNet and a BERT servable co-resident on
one MI355X behind the native transport, Predicts to both in flight through the
reference-shaped client, and HandleReloadConfigRequest hot reloads that drop
and re-add BERT while ResNet traffic continues (model_service.proto:19-21: the
new config supersedes the old one)."""
import asyncio
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

from rust_tensorflow_serving2_amd.client import ModelDescription, TensorflowServing, TFServingError  # noqa: E402
from rust_tensorflow_serving2_amd.schema import serving  # noqa: E402
from rust_tensorflow_serving2_amd.server.servable import ServableOptions  # noqa: E402
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions  # noqa: E402


@pytest.fixture(scope="module")
def paths(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import bert, resnet
    root = tmp_path_factory.mktemp("mm")
    rpath = str(root / "resnet")
    bpath = str(root / "bert")
    resnet.export(os.path.join(rpath, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=10, image_size=32, seed=3)
    bert.export(os.path.join(bpath, "1"), bert.BertConfig(vocab_size=1000, hidden=128, layers=2, heads=2,
                                                         intermediate=256, seq_len=64), seed=4)
    return rpath, bpath


def _config(*models):
    cfg = serving.ModelServerConfig()
    for name, path in models:
        cfg.model_config_list.config.add(name=name, base_path=path, model_platform="tensorflow")
    return cfg


def _bert_feeds(rng, n=2):
    ids = rng.integers(0, 1000, (n, 64)).astype(np.int32)
    return {"input_ids": ids, "input_mask": np.ones((n, 64), np.int32), "segment_ids": np.zeros((n, 64), np.int32)}


def test_resnet_and_bert_coresident_with_hot_reload(paths):
    rpath, bpath = paths
    so = ServableOptions(device="cuda:0", max_batch_size=8, allowed_batch_sizes=(1, 2, 4, 8))
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_config=_config(("resnet", rpath), ("bert", bpath)),
                                    device="cuda:0", transport="native", servable=so,
                                    file_system_poll_wait_seconds=0, batch_timeout_us=500)).start()
    rng = np.random.default_rng(0)
    img = rng.random((1, 32, 32, 3), dtype=np.float32)

    async def scenario():
        cl = await TensorflowServing.new().hostname("127.0.0.1").port(srv.port).build()
        ref_r = await cl.predict_tensors("resnet", {"input": img})
        ref_b = await cl.predict_tensors("bert", _bert_feeds(np.random.default_rng(1)))
        assert ref_r["probabilities"].shape == (1, 10)
        assert ref_b["probabilities"].shape[0] == 2

        # concurrent traffic to both models on one shared channel
        rs = await asyncio.gather(*[cl.predict_tensors("resnet", {"input": img}) for _ in range(16)],
                                  *[cl.predict_tensors("bert", _bert_feeds(np.random.default_rng(1)))
                                    for _ in range(8)])
        for r in rs[:16]:
            np.testing.assert_allclose(r["probabilities"], ref_r["probabilities"], atol=1e-3)
        for r in rs[16:]:
            np.testing.assert_allclose(r["probabilities"], ref_b["probabilities"], atol=1e-3)

        # reload to {resnet} while resnet requests are in flight: they all succeed,
        # bert goes away
        inflight = [asyncio.ensure_future(cl.predict_tensors("resnet", {"input": img})) for _ in range(32)]
        resp = await cl.reload(_config(("resnet", rpath)).model_config_list.config[0])
        assert resp.status.error_code == 0
        for r in await asyncio.gather(*inflight):
            np.testing.assert_allclose(r["probabilities"], ref_r["probabilities"], atol=1e-3)
        with pytest.raises(TFServingError):
            await cl.predict_tensors("bert", _bert_feeds(np.random.default_rng(1)))
        st = await cl.model_status(ModelDescription("resnet"))
        assert st.model_version_status[0].state == serving.ModelVersionStatus.AVAILABLE

        # reload back to both: bert serves again with the same numerics
        cfg = _config(("resnet", rpath), ("bert", bpath))
        resp = await cl.reload(list(cfg.model_config_list.config))
        assert resp.status.error_code == 0
        for _ in range(200):
            try:
                again = await cl.predict_tensors("bert", _bert_feeds(np.random.default_rng(1)))
                break
            except TFServingError:
                await asyncio.sleep(0.05)
        else:
            raise AssertionError("bert did not come back after the reload")
        np.testing.assert_allclose(again["probabilities"], ref_b["probabilities"], atol=1e-3)
        r = await cl.predict_tensors("resnet", {"input": img})
        np.testing.assert_allclose(r["probabilities"], ref_r["probabilities"], atol=1e-3)

    try:
        asyncio.run(scenario())
    finally:
        srv.stop()


def test_unloading_a_model_answers_its_in_flight_requests(paths):
    """Reload to a config WITHOUT the model that has Predicts in flight on the
    fast path (batched into slots, queued, or still streaming): every call gets
    an answer -- its result or UNAVAILABLE / NOT_FOUND -- and none waits for its
    deadline (batcher.cpp Endpoint::close)."""
    import time
    import grpc
    from rust_tensorflow_serving2_amd import native
    rpath, _bpath = paths
    so = ServableOptions(device="cuda:0", max_batch_size=8, allowed_batch_sizes=(1, 2, 4, 8))
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1",
                                    model_config=_config(("keep", rpath), ("gone", rpath)),
                                    device="cuda:0", transport="native", servable=so,
                                    file_system_poll_wait_seconds=0, batch_timeout_us=2000)).start()
    try:
        tr = srv.transports[0]
        for _ in range(400):
            if len(tr.stats().get("endpoints", [])) >= 2:
                break
            time.sleep(0.05)
        img = np.random.default_rng(5).random((1, 32, 32, 3), dtype=np.float32)
        body = native.encode_predict_request(native.spec_tuple("gone", None, None, ""), {"input": img})

        async def scenario():
            async with grpc.aio.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
                stub = ch.unary_unary("/tensorflow.serving.PredictionService/Predict")
                calls = [asyncio.ensure_future(stub(body, timeout=20)) for _ in range(96)]
                await asyncio.sleep(0.01)
                cl = await TensorflowServing.new().hostname("127.0.0.1").port(srv.port).build()
                resp = await cl.reload(_config(("keep", rpath)).model_config_list.config[0])
                assert resp.status.error_code == 0
                t0 = time.time()
                codes = []
                for c in calls:
                    try:
                        await c
                        codes.append("OK")
                    except grpc.aio.AioRpcError as e:
                        codes.append(e.code().name)
                return codes, time.time() - t0
        codes, waited = asyncio.run(scenario())
        assert len(codes) == 96 and "DEADLINE_EXCEEDED" not in codes, codes
        assert set(codes) <= {"OK", "UNAVAILABLE", "NOT_FOUND"}, set(codes)
        assert waited < 15
    finally:
        srv.stop()
