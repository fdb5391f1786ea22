"""Native HTTP/2 front end: wire interop with grpcio's C-core client, error
statuses, concurrency, and the native load generator (CPU, half_plus_two)."""
import asyncio

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import _C, native
from rust_tensorflow_serving2_amd.client import TensorflowServing, TFServingError, unpack_signature_defs
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions

import grpc


@pytest.fixture(scope="module")
def nserver(hpt_path):
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="hpt", model_base_path=hpt_path,
                                    transport="native", file_system_poll_wait_seconds=0)).start()
    yield srv
    srv.stop()


def test_grpcio_client_interop(nserver):
    async def go():
        c = await TensorflowServing.new().hostname("127.0.0.1").port(nserver.port).build()
        st = await c.model_status("hpt")
        assert st.model_version_status[0].state == 30
        assert "serving_default" in unpack_signature_defs(await c.model_metadata("hpt"))
        out = await c.predict_tensors("hpt", {"x": np.array([[1.0], [3.0]], np.float32)})
        np.testing.assert_allclose(out["y"].reshape(-1), [2.5, 3.5])
        with pytest.raises(TFServingError) as ei:
            await c.model_status("missing")
        assert ei.value.code == grpc.StatusCode.NOT_FOUND
        res = await asyncio.gather(*[c.clone().predict_tensors("hpt", {"x": np.full((1, 1), i, np.float32)})
                                     for i in range(40)])
        np.testing.assert_allclose([r["y"][0, 0] for r in res], [0.5 * i + 2 for i in range(40)])
        await c.close()
    asyncio.run(go())


def test_unknown_method_and_large_message(nserver):
    async def go():
        ch = grpc.aio.insecure_channel(f"127.0.0.1:{nserver.port}",
                                       options=[("grpc.max_send_message_length", 64 << 20),
                                                ("grpc.max_receive_message_length", 64 << 20)])
        with pytest.raises(grpc.aio.AioRpcError) as ei:
            await ch.unary_unary("/tensorflow.serving.PredictionService/Nope")(b"")
        assert ei.value.code() == grpc.StatusCode.UNIMPLEMENTED
        # 20 MB request (a client-side batch of 32 images) is accepted (raised limits)
        x = np.zeros((5_000_000, 1), np.float32)
        body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": x})
        raw = await ch.unary_unary("/tensorflow.serving.PredictionService/Predict")(body)
        assert len(raw) > 20_000_000
        await ch.close()
    asyncio.run(go())


def test_native_loadgen(nserver):
    body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": np.ones((1, 1), np.float32)})
    r = _C.run_loadgen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [body],
                       300, 16, 4, 2, 60.0)
    assert r["ok"] == 300 and r["errors"] == 0, r["first_error"]
    assert len(r["latency_us"]) == 300
    bad = native.encode_predict_request(native.spec_tuple("nope", None, None, ""), {"x": np.ones((1, 1), np.float32)})
    r = _C.run_loadgen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [bad],
                       10, 4, 1, 1, 60.0)
    assert r["errors"] == 10 and "grpc-status 5" in r["first_error"]


def test_persistent_loadgen_reuses_connections(nserver):
    """LoadGen opens its HTTP/2 connections once; repeated runs (warmup, then
    the timed window in bench.py) reuse them and count only their own calls."""
    body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": np.ones((3, 1), np.float32)})
    lg = _C.LoadGen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [body], 16, 4, 2)
    assert lg.run(1, 60.0)["ok"] == 1     # every connection accepted by now
    before = nserver.transports[0].stats()["connections"]
    for n in (50, 200, 7):
        r = lg.run(n, 60.0)
        assert r["ok"] == n and r["errors"] == 0, r["first_error"]
        assert len(r["latency_us"]) == n
    assert nserver.transports[0].stats()["connections"] == before   # no new connections per run
    del lg


def test_connections_spread_evenly_over_io_threads(nserver):
    """One acceptor hands each connection to the IO thread with the fewest
    live connections: the reference client's two connections always land on
    two threads (the per-thread SO_REUSEPORT hash put both on one thread in
    about one run in six), and eight connections fill four threads evenly."""
    import time
    srv = nserver.transports[0].srv

    def settled():
        prev = None
        for _ in range(40):
            cur = srv.stats()["io_connections"]
            if cur == prev:
                return cur
            prev = cur
            time.sleep(0.05)
        return prev
    body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": np.ones((1, 1), np.float32)})
    base = settled()
    assert len(base) >= 2
    lg2 = _C.LoadGen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [body], 4, 2, 2)
    assert lg2.run(4, 60.0)["ok"] == 4
    two = settled()
    grew = [b - a for a, b in zip(base, two)]
    if max(base) == min(base):
        assert sorted(grew)[-2:] == [1, 1], (base, two)     # two threads, one connection each
    lg8 = _C.LoadGen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [body], 16, 8, 2)
    assert lg8.run(16, 60.0)["ok"] == 16
    eight = settled()
    assert sum(eight) == sum(two) + 8
    assert max(eight) - min(eight) <= max(1, max(two) - min(two)), (two, eight)
    del lg2, lg8


def test_continuous_loadgen_windows(nserver):
    """bench.py's steady-state mode: the load generator keeps `concurrency`
    calls in flight from start() to stop(); each window counts exactly its own
    n completions (latency per completion), whatever n is."""
    body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": np.ones((2, 1), np.float32)})
    lg = _C.LoadGen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", [body], 16, 4, 2)
    lg.start()
    done0 = lg.completed()
    for n in (5, 100, 1, 37):
        r = lg.window(n, 60.0)
        assert r["ok"] == n and r["errors"] == 0, r["first_error"]
        assert len(r["latency_us"]) == n and min(r["latency_us"]) > 0
        assert r["elapsed_s"] > 0
    assert lg.completed() >= done0 + 143
    tot = lg.stop(30.0)
    assert tot["errors"] == 0 and tot["ok"] >= 143
    with pytest.raises(RuntimeError):
        lg.window(1, 1.0)             # needs start()
    assert lg.run(10, 60.0)["ok"] == 10   # the connections stay usable for batch runs
    lg.start()
    assert lg.window(20, 60.0)["ok"] == 20
    del lg                            # destructor stops a running generator


def test_native_loadgen_large_bodies(nserver):
    """Multi-frame (zero-copy DATA) requests of different sizes on shared connections."""
    bodies = [native.encode_predict_request(native.spec_tuple("hpt", None, None, ""),
                                            {"x": np.full((n, 1), float(n), np.float32)})
              for n in (50_000, 150_528, 7, 300_000)]
    r = _C.run_loadgen("127.0.0.1", nserver.port, "/tensorflow.serving.PredictionService/Predict", bodies,
                       64, 16, 3, 2, 120.0)
    assert r["ok"] == 64 and r["errors"] == 0, r["first_error"]
    assert r["bytes_sent"] >= 64 * min(len(b) for b in bodies)


def test_native_counters_in_prometheus_metrics(hpt_path):
    import json
    import urllib.request
    srv = ModelServer(ServerOptions(port=0, rest_api_port=-1, host="127.0.0.1", model_name="hpt",
                                    model_base_path=hpt_path, transport="native",
                                    file_system_poll_wait_seconds=0)).start()
    try:
        body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""),
                                             {"x": np.ones((1, 1), np.float32)})
        r = _C.run_loadgen("127.0.0.1", srv.port, "/tensorflow.serving.PredictionService/Predict", [body],
                           20, 4, 1, 1, 60.0)
        assert r["ok"] == 20
        with urllib.request.urlopen(f"http://127.0.0.1:{srv.rest_port}/monitoring/prometheus/metrics") as f:
            text = f.read().decode()
        assert 'tfserve_native_requests_total{kind="requests"} 20' in text
        assert 'tfserve_native_io_seconds_total{phase="recv"}' in text
    finally:
        srv.stop()


def test_trace_dir_records_rpcs(hpt_path, tmp_path, monkeypatch):
    """Per-RPC trace records of the Python core (the CPU fast path, which
    batches in C++, is switched off so every call takes the traced path)."""
    from rust_tensorflow_serving2_amd.server import native_transport
    from rust_tensorflow_serving2_amd.utils import tracing
    monkeypatch.setattr(native_transport, "CPU_FAST_PATH", False)
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="hpt", model_base_path=hpt_path,
                                    transport="native", file_system_poll_wait_seconds=0,
                                    trace_dir=str(tmp_path / "tr"))).start()
    try:
        body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""),
                                             {"x": np.ones((1, 1), np.float32)})
        assert _C.run_loadgen("127.0.0.1", srv.port, "/tensorflow.serving.PredictionService/Predict", [body],
                              10, 2, 1, 1, 60.0)["ok"] == 10
    finally:
        srv.stop()
    recs = tracing.load(srv.tracer.path)
    rpcs = [r for r in recs if r["type"] == "rpc"]
    assert len(rpcs) == 10 and all(r["end_us"] >= r["start_us"] for r in rpcs)
    chrome = tracing.to_chrome(recs)
    assert len(chrome["traceEvents"]) == 10


def test_cpu_servable_rides_the_batched_fast_path(hpt_path):
    """BASELINE config 1 (half_plus_two on CPU): requests are decoded, batched
    and answered in C++; Python runs the CPU program once per batch
    (server/cpu_runtime.py).  Results equal the per-request Python path."""
    import concurrent.futures as cf
    import grpc
    from rust_tensorflow_serving2_amd.schema import serving
    from rust_tensorflow_serving2_amd.utils import tensors as T
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="hpt", model_base_path=hpt_path,
                                    transport="native", file_system_poll_wait_seconds=0,
                                    batch_timeout_us=1000)).start()
    try:
        tr = srv.transports[0]
        import time
        for _ in range(200):
            if tr.stats().get("endpoints"):
                break
            time.sleep(0.02)
        assert tr.stats()["endpoints"], "no fast-path endpoint for the CPU servable"
        xs = [np.array([[float(i)], [float(i) + 0.5]], np.float32) for i in range(64)]
        bodies = [native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": x}) for x in xs]
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            stub = ch.unary_unary("/tensorflow.serving.PredictionService/Predict")
            with cf.ThreadPoolExecutor(16) as ex:
                outs = list(ex.map(lambda b: stub(b, timeout=30), bodies))
        for x, raw in zip(xs, outs):
            y = T.tensor_proto_to_numpy(serving.PredictResponse.FromString(raw).outputs["y"])
            np.testing.assert_allclose(y, x * 0.5 + 2.0, rtol=1e-6)
        st = tr.srv.stats()
        assert st["fast_path"] == 64 and st["slow_path"] == 0, st
        eps = list(tr.stats()["endpoints"].values())
        assert sum(e["rows"] for e in eps) == 128 and sum(e["batches"] for e in eps) < 64   # batched
        r = _C.run_loadgen("127.0.0.1", srv.port, "/tensorflow.serving.PredictionService/Predict", bodies[:8],
                           2000, 32, 2, 2, 60.0)
        assert r["ok"] == 2000 and r["errors"] == 0
    finally:
        srv.stop()
