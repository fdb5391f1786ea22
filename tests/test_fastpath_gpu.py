"""Native Predict fast path on the GPU: results must equal the Python slow path
(same servable), partial batches / mixed request batch sizes / output_filter,
and fall-through for requests the fast path does not take (labels, bad shapes)."""
import asyncio
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

import grpc  # noqa: E402

from rust_tensorflow_serving2_amd import _C, native  # noqa: E402
from rust_tensorflow_serving2_amd.schema import serving  # noqa: E402
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions  # noqa: E402
from rust_tensorflow_serving2_amd.server.servable import ServableOptions  # noqa: E402

PREDICT = "/tensorflow.serving.PredictionService/Predict"


@pytest.fixture(scope="module")
def gpu_server(tmp_path_factory):
    from rust_tensorflow_serving2_amd.models import resnet
    base = str(tmp_path_factory.mktemp("fp") / "resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=10, image_size=32, seed=5)
    so = ServableOptions(device="cuda:0", max_batch_size=8, allowed_batch_sizes=(1, 2, 4, 8))
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="resnet", model_base_path=base,
                                    device="cuda:0", transport="native", servable=so,
                                    file_system_poll_wait_seconds=0, batch_timeout_us=500)).start()
    tr = srv.transports[0]
    import time
    for _ in range(300):
        if tr.stats().get("endpoints"):
            break
        time.sleep(0.05)
    assert tr.stats()["endpoints"], "fast path endpoint not registered"
    yield srv
    srv.stop()


def _call(port, body):
    async def go():
        async with grpc.aio.insecure_channel(f"127.0.0.1:{port}") as ch:
            return await ch.unary_unary(PREDICT)(body)
    return asyncio.run(go())


def test_fast_path_matches_slow_path(gpu_server):
    x = np.random.default_rng(0).random((3, 32, 32, 3), dtype=np.float32)
    spec = native.spec_tuple("resnet", None, None, "serving_default")
    fast = serving.PredictResponse.FromString(_call(gpu_server.port, native.encode_predict_request(spec, {"input": x})))
    slow = serving.PredictResponse.FromString(
        gpu_server.core.predict(native.encode_predict_request(spec, {"input": x})))
    for k in ("probabilities", "classes"):
        a = np.array(fast.outputs[k].float_val or fast.outputs[k].int64_val)
        b = np.array(slow.outputs[k].float_val or slow.outputs[k].int64_val)
        np.testing.assert_allclose(a, b, atol=2e-4)
    assert fast.model_spec.version.value == 1 and fast.model_spec.signature_name == "serving_default"
    assert list(d.size for d in fast.outputs["probabilities"].tensor_shape.dim) == [3, 10]
    st = gpu_server.transports[0].stats()
    assert st["fast_path"] >= 1


def test_many_concurrent_rows_are_routed_back_correctly(gpu_server):
    """Each request gets ITS rows back even when batched with others."""
    rng = np.random.default_rng(1)
    xs = [rng.random((1 + (i % 3), 32, 32, 3), dtype=np.float32) for i in range(24)]
    spec = native.spec_tuple("resnet", None, None, "")
    bodies = [native.encode_predict_request(spec, {"input": x}) for x in xs]

    async def go():
        async with grpc.aio.insecure_channel(f"127.0.0.1:{gpu_server.port}") as ch:
            stub = ch.unary_unary(PREDICT)
            return await asyncio.gather(*[stub(b) for b in bodies])
    outs = asyncio.run(go())
    for x, raw in zip(xs, outs):
        ref = serving.PredictResponse.FromString(
            gpu_server.core.predict(native.encode_predict_request(spec, {"input": x})))
        got = np.array(serving.PredictResponse.FromString(raw).outputs["probabilities"].float_val)
        np.testing.assert_allclose(got, np.array(ref.outputs["probabilities"].float_val), atol=2e-4)


def test_output_filter_and_fallthrough(gpu_server):
    x = np.random.default_rng(2).random((1, 32, 32, 3), dtype=np.float32)
    body = native.encode_predict_request(native.spec_tuple("resnet", 1, None, "serving_default"), {"input": x},
                                         ["classes"])
    r = serving.PredictResponse.FromString(_call(gpu_server.port, body))
    assert list(r.outputs) == ["classes"]
    # wrong image size -> not fast-pathable -> python path returns INVALID_ARGUMENT
    bad = native.encode_predict_request(native.spec_tuple("resnet", None, None, ""),
                                        {"input": np.zeros((1, 31, 32, 3), np.float32)})
    with pytest.raises(grpc.aio.AioRpcError) as ei:
        _call(gpu_server.port, bad)
    assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT


def test_loadgen_against_fast_path(gpu_server):
    spec = native.spec_tuple("resnet", None, None, "")
    bodies = [native.encode_predict_request(spec, {"input": np.random.default_rng(i).random((1, 32, 32, 3),
                                                                                           dtype=np.float32)})
              for i in range(8)]
    r = _C.run_loadgen("127.0.0.1", gpu_server.port, PREDICT, bodies, 400, 32, 4, 2, 120.0)
    assert r["ok"] == 400 and r["errors"] == 0, r["first_error"]


def test_native_lanes_and_injected_faults(tmp_path, monkeypatch):
    """Native C++ lanes serve the batches; an injected lane fault fails only the
    requests of that batch (INTERNAL) and the server keeps serving."""
    from rust_tensorflow_serving2_amd.models import resnet
    import time
    monkeypatch.setenv("TFSERVE_FAULT", "lane_every=3")
    base = str(tmp_path / "resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=10, image_size=32, seed=6)
    so = ServableOptions(device="cuda:0", max_batch_size=4, allowed_batch_sizes=(1, 2, 4), lanes=1)
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="resnet", model_base_path=base,
                                    device="cuda:0", transport="native", servable=so,
                                    file_system_poll_wait_seconds=0, batch_timeout_us=200,
                                    trace_dir=str(tmp_path / "trace"))).start()
    try:
        tr = srv.transports[0]
        for _ in range(300):
            if tr.stats().get("endpoints"):
                break
            time.sleep(0.05)
        eps = list(tr._eps.values())
        assert eps and eps[0].native_lanes == 1
        x = np.random.default_rng(7).random((1, 32, 32, 3), dtype=np.float32)
        body = native.encode_predict_request(native.spec_tuple("resnet", None, None, ""), {"input": x})
        codes = []
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            stub = ch.unary_unary(PREDICT)
            for _ in range(9):                       # sequential: one request per batch
                try:
                    stub(body, timeout=30)
                    codes.append("OK")
                except grpc.RpcError as e:
                    assert "injected fault" in e.details()
                    codes.append(e.code().name)
        assert codes.count("INTERNAL") == 3 and codes.count("OK") == 6, codes
        stats = srv.transports[0].srv.native_lane_stats()
        assert stats and sum(s[2] for s in stats) == 3
    finally:
        srv.stop()
    from rust_tensorflow_serving2_amd.utils import tracing
    batches = [r for r in tracing.load(srv.tracer.path) if r["type"] == "batch"]
    assert len(batches) == 6        # the 6 successful batches (faulted ones are not traced)
    assert all(r["opened_us"] <= r["acquired_us"] <= r["done_us"] <= r["posted_us"] for r in batches)


def test_native_lane_device_failure_reloads_servable(tmp_path, monkeypatch):
    """A native lane whose every batch fails after the first 2 (lane_after=2,
    a device gone bad) trips the health monitor through the endpoint's
    consecutive-failure counter; the version is unloaded and loaded again and
    serves OK afterwards (server/health.py)."""
    from rust_tensorflow_serving2_amd.models import resnet
    import time
    monkeypatch.setenv("TFSERVE_FAULT", "lane_after=2")
    base = str(tmp_path / "resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=10, image_size=32, seed=6)
    so = ServableOptions(device="cuda:0", max_batch_size=4, allowed_batch_sizes=(1, 2, 4), lanes=1)
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="resnet", model_base_path=base,
                                    device="cuda:0", transport="native", servable=so,
                                    file_system_poll_wait_seconds=0, batch_timeout_us=200,
                                    health_failure_threshold=3, health_max_recoveries=10)).start()
    try:
        tr = srv.transports[0]
        for _ in range(300):
            if tr.stats().get("endpoints"):
                break
            time.sleep(0.05)
        x = np.random.default_rng(7).random((1, 32, 32, 3), dtype=np.float32)
        body = native.encode_predict_request(native.spec_tuple("resnet", None, None, ""), {"input": x})
        codes = []
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            stub = ch.unary_unary(PREDICT)
            for _ in range(80):
                try:
                    stub(body, timeout=30)
                    codes.append("OK")
                except grpc.RpcError as e:
                    codes.append(e.code().name)
                if srv.health.recoveries.get(("resnet", 1), 0) >= 1 and "OK" in codes[codes.index("INTERNAL"):]:
                    break
                time.sleep(0.05)
        assert codes[:2] == ["OK", "OK"], codes
        assert srv.health.recoveries.get(("resnet", 1), 0) >= 1, codes
        assert "OK" in codes[codes.index("INTERNAL"):], codes      # served again after the reload
        assert srv.health.failures[("resnet", 1)] >= 3
    finally:
        srv.stop()


@pytest.mark.parametrize("ingest", ["bf16", "fp32"])
def test_request_logging_on_the_gpu_fast_path(tmp_path, monkeypatch, ingest):
    """logging_config sampling_rate=1.0 on a GPU model: every Predict served by
    the native fast path (streamed 300 KB images included) is read back as a
    valid PredictionLog TFRecord holding the request as sent and the response
    as received.  With bf16 ingest a row no longer holds the request's fp32
    bytes, so a logged endpoint buffers those requests instead of streaming."""
    monkeypatch.setenv("TFSERVE_BF16_INGEST", "1" if ingest == "bf16" else "0")
    from rust_tensorflow_serving2_amd.models import resnet
    from rust_tensorflow_serving2_amd.utils.request_log import read_tfrecords
    import time
    base = str(tmp_path / "resnet")
    resnet.export(os.path.join(base, "1"), blocks=(1, 1, 1, 1), width=16, num_classes=10, image_size=160, seed=8)
    cfg = serving.ModelServerConfig()
    mc = cfg.model_config_list.config.add(name="resnet", base_path=base, model_platform="tensorflow")
    mc.logging_config.log_collector_config.filename_prefix = str(tmp_path / "logs" / "resnet")
    mc.logging_config.sampling_config.sampling_rate = 1.0
    so = ServableOptions(device="cuda:0", max_batch_size=4, allowed_batch_sizes=(1, 2, 4))
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_config=cfg, device="cuda:0", transport="native",
                                    servable=so, file_system_poll_wait_seconds=0, batch_timeout_us=300)).start()
    try:
        tr = srv.transports[0]
        for _ in range(300):
            if tr.stats().get("endpoints"):
                break
            time.sleep(0.05)
        assert tr.stats()["endpoints"]
        rng = np.random.default_rng(9)
        spec = native.spec_tuple("resnet", None, None, "")
        bodies = [native.encode_predict_request(spec, {"input": rng.random((1 + i % 2, 160, 160, 3),
                                                                           dtype=np.float32)})
                  for i in range(12)]

        async def go():
            async with grpc.aio.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
                stub = ch.unary_unary(PREDICT)
                return await asyncio.gather(*[stub(b) for b in bodies])
        outs = asyncio.run(go())
        st = tr.srv.stats()
        assert st["fast_path"] == 12 and st["slow_path"] == 0, st
        assert (st["streamed"] == 0) if ingest == "bf16" else (st["streamed"] >= 1), st
        lg = srv.request_logs.get("resnet")
        lg.flush()
        recs = [serving.PredictionLog.FromString(r) for r in read_tfrecords(lg.path)]
        assert len(recs) == 12
        sent = dict(zip(bodies, outs))
        for pl in recs:
            req = pl.predict_log.request.SerializeToString()
            if req not in sent:
                same = [b for b in sent if len(b) == len(req)]
                diffs = [next(i for i, (x, y) in enumerate(zip(b, req)) if x != y) for b in same]
                raise AssertionError(f"logged request ({len(req)} B) matches no sent body; first differing "
                                     f"offsets vs the {len(same)} same-length bodies: {diffs}")
            # compare as messages: map entries (the outputs) have no canonical wire order, and
            # the re-serialised log copy need not list them in the order the server sent them
            assert pl.predict_log.response == serving.PredictResponse.FromString(sent[req])
            assert pl.log_metadata.model_spec.name == "resnet" and pl.log_metadata.model_spec.version.value == 1
        assert lg.stats()["dropped"] == 0
    finally:
        srv.stop()


