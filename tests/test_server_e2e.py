"""End-to-end over real gRPC (BASELINE config 1: half_plus_two on CPU): every
RPC of the wire contract through the reference-shaped client, error codes,
concurrency on one channel (examples/async.rs pattern), hot reload semantics."""
import asyncio
import os
import shutil

import numpy as np
import pytest

from rust_tensorflow_serving2_amd.client import (ModelDescription, TensorflowServing, TFServingError,
                                                 unpack_signature_defs)
from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions

import grpc


@pytest.fixture(scope="module")
def server(hpt_path, tiny_resnet_path):
    cfg = serving.ModelServerConfig()
    for name, path in (("half_plus_two", hpt_path), ("resnet", tiny_resnet_path)):
        mc = cfg.model_config_list.config.add(name=name, base_path=path, model_platform="tensorflow")
    srv = ModelServer(ServerOptions(port=0, model_config=cfg, file_system_poll_wait_seconds=0.2)).start()
    yield srv
    srv.stop()


def run(coro):
    return asyncio.run(coro)


async def client(port, sig=None):
    b = TensorflowServing.new().hostname("127.0.0.1").port(port)
    if sig:
        b = b.signature_name(sig)
    return await b.build()


def test_builder_errors():
    async def go():
        with pytest.raises(TFServingError, match="hostname not provided"):
            await TensorflowServing.new().port(1).build()
        with pytest.raises(TFServingError, match="port not provided"):
            await TensorflowServing.new().hostname("x").build()
    run(go())


def test_predict_half_plus_two(server):
    async def go():
        c = await client(server.port)
        out = await c.predict_tensors("half_plus_two", {"x": np.array([[1.0], [2.0], [5.0]], np.float32)})
        np.testing.assert_allclose(out["y"].reshape(-1), [2.5, 3.0, 4.5])
        raw = await c.predict_tensors(ModelDescription("half_plus_two", 1),
                                      {"x": np.array([[1.0]], np.float32)}, raw=True)
        resp = serving.PredictResponse.FromString(raw)
        assert resp.model_spec.name == "half_plus_two" and resp.model_spec.version.value == 1
        assert resp.model_spec.signature_name == "serving_default"
    run(go())


def test_predict_resnet_image(server, tmp_path):
    from PIL import Image
    img = Image.fromarray((np.random.default_rng(0).random((32, 32, 3)) * 255).astype(np.uint8))
    path = tmp_path / "cat.png"
    img.save(path)

    async def go():
        c = await client(server.port)
        resp = await c.predict_with_preprocessing(str(path), "resnet", lambda v: v / 255.0)
        probs = np.array(resp.outputs["probabilities"].float_val).reshape(1, 11)
        assert abs(probs.sum() - 1) < 1e-4
        assert resp.outputs["classes"].int64_val[0] == int(probs.argmax())
        # same image through predict() (identity preprocessing) also works
        await c.predict(img, "resnet")
    run(go())


def test_metadata_and_status(server):
    async def go():
        c = await client(server.port)
        st = await c.model_status("half_plus_two")
        assert [(s.version, s.state) for s in st.model_version_status] == [(1, 30)]
        md = await c.model_metadata("resnet")
        sigs = unpack_signature_defs(md)
        assert set(sigs) == {"serving_default", "predict"}
        assert sigs["serving_default"].inputs["input"].name == "input_tensor:0"
        assert md.model_spec.version.value == 1
    run(go())


def test_classify_regress_multi(server):
    async def go():
        c = await client(server.port, "classify_x_to_y")
        res = await c.classify("half_plus_two", {"x": [3.0]})
        assert res.classifications[0].classes[0].score == pytest.approx(3.5)
        r = await client(server.port, "regress_x_to_y")
        res = await r.regress("half_plus_two", {"x": [4.0]})
        assert res.regressions[0].value == pytest.approx(4.0)
        mi = await c.multi_inference("half_plus_two", [("regress_x_to_y", "tensorflow/serving/regress"),
                                                       ("classify_x_to_y", "tensorflow/serving/classify")],
                                     {"x": [1.0]})
        assert mi.results[0].regression_result.regressions[0].value == pytest.approx(2.5)
        assert mi.results[1].classification_result.classifications[0].classes[0].score == pytest.approx(2.5)
    run(go())


@pytest.mark.parametrize("call,code", [
    (lambda c: c.model_status("nope"), grpc.StatusCode.NOT_FOUND),
    (lambda c: c.predict_tensors("nope", {"x": np.zeros((1, 1), np.float32)}), grpc.StatusCode.NOT_FOUND),
    (lambda c: c.predict_tensors(ModelDescription("half_plus_two", 9), {"x": np.zeros((1, 1), np.float32)}),
     grpc.StatusCode.NOT_FOUND),
    (lambda c: c.predict_tensors("half_plus_two", {"bogus": np.zeros((1, 1), np.float32)}),
     grpc.StatusCode.INVALID_ARGUMENT),
    (lambda c: c.predict_tensors("half_plus_two", {"x": np.zeros((1, 1), np.int64)}),
     grpc.StatusCode.INVALID_ARGUMENT),
    (lambda c: c.predict_tensors("half_plus_two", {"x": np.zeros((1, 1), np.float32)}, ["nope"]),
     grpc.StatusCode.INVALID_ARGUMENT),
    (lambda c: c.classify("half_plus_two", {"x": [1.0]}), grpc.StatusCode.INVALID_ARGUMENT),
])
def test_error_codes(server, call, code):
    async def go():
        c = await client(server.port)
        with pytest.raises(TFServingError) as ei:
            await call(c)
        assert ei.value.code == code
    run(go())


def test_concurrent_clones_share_channel(server):
    async def go():
        c = await client(server.port)
        futs = []
        for i in range(16):
            s = c.clone()
            futs.append(s.model_status("half_plus_two"))
            futs.append(s.model_metadata("half_plus_two"))
            futs.append(s.predict_tensors("half_plus_two", {"x": np.full((1, 1), i, np.float32)}))
        res = await asyncio.gather(*futs)
        ys = [r["y"][0, 0] for r in res[2::3]]
        np.testing.assert_allclose(ys, [0.5 * i + 2 for i in range(16)])
    run(go())


def test_new_version_polling_and_labels(server, hpt_path, tmp_path):
    base = str(tmp_path / "hpt")
    shutil.copytree(os.path.join(hpt_path, "1"), os.path.join(base, "1"))

    async def go():
        c = await client(server.port)
        mc = serving.ModelConfig(name="hpt_poll", base_path=base, model_platform="tensorflow")
        mc.model_version_policy.all.SetInParent()
        keep = [serving.ModelConfig(name="half_plus_two", base_path=hpt_path, model_platform="tensorflow"),
                serving.ModelConfig(name="resnet", base_path=server.manager.model_config("resnet").base_path,
                                    model_platform="tensorflow"), mc]
        r = await c.reload(keep)
        assert r.status.error_code == 0
        shutil.copytree(os.path.join(base, "1"), os.path.join(base, "2"))
        for _ in range(100):
            st = await c.model_status("hpt_poll")
            if len([s for s in st.model_version_status if s.state == 30]) == 2:
                break
            await asyncio.sleep(0.1)
        assert sorted(s.version for s in st.model_version_status if s.state == 30) == [1, 2]
        # latest routing picks version 2
        raw = await c.predict_tensors("hpt_poll", {"x": np.ones((1, 1), np.float32)}, raw=True)
        assert serving.PredictResponse.FromString(raw).model_spec.version.value == 2
        # version labels
        mc.version_labels["stable"] = 1
        r = await c.reload(keep[:2] + [mc])
        assert r.status.error_code == 0
        req = serving.GetModelStatusRequest()
        req.model_spec.name = "hpt_poll"
        req.model_spec.version_label = "stable"
        st = serving.GetModelStatusResponse.FromString(server.core.get_model_status(req.SerializeToString()))
        assert [s.version for s in st.model_version_status] == [1]
        # reload without the model: it is unloaded (model_service.proto:19-21)
        r = await c.reload(keep[:2])
        for _ in range(50):
            st = await c.model_status("hpt_poll")
            if all(s.state == 50 for s in st.model_version_status):
                break
            await asyncio.sleep(0.1)
        assert all(s.state == 50 for s in st.model_version_status)
        # bad base path: reported in the response status, server keeps serving others
        r = await c.reload(keep[:2] + [serving.ModelConfig(name="bad", base_path="/nonexistent")])
        assert r.status.error_code == 5
        out = await c.predict_tensors("half_plus_two", {"x": np.ones((1, 1), np.float32)})
        assert out["y"][0, 0] == 2.5
    run(go())
