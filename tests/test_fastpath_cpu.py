"""The C++ Predict fast path without a GPU: a Python thread plays the GPU lane
(acquire -> compute on the slot buffers -> complete) so the batcher, the
streaming decode (payload copied socket -> slot row as DATA frames arrive),
the buffered fallback and the FIFO queue are exercised on CPU."""
import concurrent.futures as cf
import threading
import time

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import _C, native
from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.utils import tensors as T

import grpc

ROW = 20000          # 80 KB of f32 per row: above the 64 KB streaming threshold
PREDICT = "/tensorflow.serving.PredictionService/Predict"


@pytest.fixture()
def fast_server():
    srv = _C.Http2Server("127.0.0.1", 0, 2)
    ep = srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [ROW])], [("y", T.DT_FLOAT, [ROW])], 8, 3000)
    slots = []
    for k in range(2):
        xin = np.zeros((8, ROW), np.float32)
        yout = np.zeros((8, ROW), np.float32)
        srv.set_slot_buffers(ep, k, [xin.ctypes.data], [yout.ctypes.data])
        slots.append((xin, yout))
    srv.set_route("m", "serving_default", -1, ep)
    srv.set_route("m", "serving_default", 1, ep)
    stop = threading.Event()
    batches = []

    def lane(k):
        xin, yout = slots[k]
        while not stop.is_set():
            n = srv.acquire(ep, k, 50)
            if n < 0:
                return
            if n == 0:
                continue
            batches.append(n)
            yout[:n] = xin[:n] * 2 + 1
            srv.complete(ep, k)

    ts = [threading.Thread(target=lane, args=(k,), daemon=True) for k in range(2)]
    srv.start()
    for t in ts:
        t.start()
    yield srv, batches
    stop.set()
    srv.remove_endpoint(ep)
    for t in ts:
        t.join(timeout=5)
    srv.stop()


def _call(port, body):
    with grpc.insecure_channel(f"127.0.0.1:{port}", options=[("grpc.max_send_message_length", 1 << 30),
                                                            ("grpc.max_receive_message_length", 1 << 30)]) as ch:
        return ch.unary_unary(PREDICT)(body, timeout=60)


def _y(raw):
    resp = serving.PredictResponse.FromString(raw)
    return T.tensor_proto_to_numpy(resp.outputs["y"])


def test_streamed_and_buffered_requests(fast_server):
    srv, batches = fast_server
    rng = np.random.default_rng(0)
    reqs = []
    for i in range(24):
        n = 1 + i % 3
        x = rng.standard_normal((n, ROW)).astype(np.float32)
        filt = ["y"] if i % 4 == 3 else []        # an output_filter after the inputs -> buffered path
        body = native.encode_predict_request(native.spec_tuple("m", None if i % 2 else 1, None, ""), {"x": x},
                                             output_filter=filt)
        reqs.append((x, body))
    # one at a time: a slot is always open, so every request without an output_filter streams
    for x, body in reqs[:8]:
        np.testing.assert_allclose(_y(_call(srv.port, body)), x * 2 + 1, rtol=1e-6)
    st = srv.stats()
    assert st["fast_path"] == 8 and st["streamed"] == 6
    assert st["direct_bytes"] > 0     # payload bytes recv()'d straight into batch rows
    # concurrently: requests that find every slot busy queue (buffered) behind the stream
    with cf.ThreadPoolExecutor(12) as ex:
        outs = list(ex.map(lambda r: _call(srv.port, r[1]), reqs[8:]))
    for (x, _b), raw in zip(reqs[8:], outs):
        np.testing.assert_allclose(_y(raw), x * 2 + 1, rtol=1e-6)
    st = srv.stats()
    assert st["fast_path"] == 24 and st["slow_path"] == 0 and st["streamed"] >= 6
    assert sum(batches) >= 24


def test_streamed_loadgen_mixed_sizes(fast_server):
    """Many multiplexed streams per connection (frames of different streams interleave)."""
    srv, _ = fast_server
    bodies = [native.encode_predict_request(native.spec_tuple("m", None, None, ""),
                                            {"x": np.full((n, ROW), n, np.float32)}) for n in (1, 2, 5, 8)]
    r = _C.run_loadgen("127.0.0.1", srv.port, PREDICT, bodies, 200, 32, 4, 2, 120.0)
    assert r["ok"] == 200 and r["errors"] == 0, r["first_error"]
    assert srv.stats()["streamed"] > 0 and srv.stats()["direct_bytes"] > 0


def test_wrong_shape_falls_back(fast_server):
    """A header the endpoint does not accept is buffered and handed to the slow path."""
    srv, _ = fast_server
    body = native.encode_predict_request(native.spec_tuple("m", None, None, ""),
                                         {"x": np.ones((1, ROW + 8), np.float32)})
    got = []

    def slow():
        c = srv.next_call(5000)
        got.append(c.body == body)
        srv.respond(c, 3, "shape mismatch", b"")
    th = threading.Thread(target=slow)
    th.start()
    with pytest.raises(grpc.RpcError) as ei:
        _call(srv.port, body)
    th.join()
    assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT and got == [True]
    assert srv.stats()["slow_path"] == 1


def test_deadline_exceeded_is_not_computed_twice():
    """A request whose grpc-timeout passes while its batch waits is answered
    DEADLINE_EXCEEDED by the batcher instead of being encoded."""
    srv = _C.Http2Server("127.0.0.1", 0, 1)
    ep = srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [ROW])], [("y", T.DT_FLOAT, [ROW])], 8, 1000)
    xin = np.zeros((8, ROW), np.float32)
    yout = np.zeros((8, ROW), np.float32)
    srv.set_slot_buffers(ep, 0, [xin.ctypes.data], [yout.ctypes.data])
    srv.set_route("m", "serving_default", -1, ep)
    stop = threading.Event()

    def slow_lane():
        while not stop.is_set():
            n = srv.acquire(ep, 0, 50)
            if n < 0:
                return
            if n > 0:
                stop.wait(0.4)               # the GPU is "busy" past the client deadline
                srv.complete(ep, 0)

    th = threading.Thread(target=slow_lane, daemon=True)
    srv.start()
    th.start()
    try:
        body = native.encode_predict_request(native.spec_tuple("m", None, None, ""), {"x": np.ones((1, ROW), np.float32)})
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            with pytest.raises(grpc.RpcError) as ei:
                ch.unary_unary(PREDICT)(body, timeout=0.15)
        assert ei.value.code() == grpc.StatusCode.DEADLINE_EXCEEDED
        deadline = time.time() + 5
        while srv.stats()["expired"] < 1 and time.time() < deadline:
            time.sleep(0.05)
        assert srv.stats()["expired"] == 1
    finally:
        stop.set()
        srv.remove_endpoint(ep)
        th.join(timeout=5)
        srv.stop()


def test_close_answers_every_unstarted_request():
    """Endpoint close (a version unloading) while requests sit in the FIFO
    queue, in an open batch and in a ready batch no lane has started: every
    one is answered (OK if its batch ran, UNAVAILABLE otherwise) -- none is
    left hanging until the client deadline."""
    srv = _C.Http2Server("127.0.0.1", 0, 2)
    ep = srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [16])], [("y", T.DT_FLOAT, [16])], 4, 1000000)
    bufs = []
    for k in range(2):
        xin, yout = np.zeros((4, 16), np.float32), np.zeros((4, 16), np.float32)
        srv.set_slot_buffers(ep, k, [xin.ctypes.data], [yout.ctypes.data])
        bufs.append((xin, yout))
    srv.set_route("m", "serving_default", -1, ep)
    started = threading.Event()

    def lane():                        # serves slot 0 once, slowly; slot 1 never runs
        while True:
            n = srv.acquire(ep, 0, 50)
            if n < 0:
                return
            if n == 0:
                continue
            started.set()
            time.sleep(0.5)
            bufs[0][1][:n] = bufs[0][0][:n] + 1
            srv.complete(ep, 0)

    def slow_path():                   # stands in for the Python core: model unloaded
        while not done.is_set():
            c = srv.next_call(50)
            if c is not None:
                srv.respond(c, 14, "Servable not found", b"")

    done = threading.Event()
    th = threading.Thread(target=lane, daemon=True)
    py = threading.Thread(target=slow_path, daemon=True)
    srv.start()
    th.start()
    py.start()
    spec = native.spec_tuple("m", None, None, "serving_default")
    body = native.encode_predict_request(spec, {"x": np.ones((1, 16), np.float32)})
    codes = []
    try:
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            stub = ch.unary_unary(PREDICT)
            with cf.ThreadPoolExecutor(16) as ex:
                futs = [ex.submit(stub, body, timeout=20) for _ in range(4)]   # fills slot 0 -> runs
                assert started.wait(5)
                futs += [ex.submit(stub, body, timeout=20) for _ in range(10)]  # slot 1 (ready) + queue
                time.sleep(0.3)
                t0 = time.time()
                srv.remove_endpoint(ep)
                for f in futs:
                    try:
                        f.result()
                        codes.append("OK")
                    except grpc.RpcError as e:
                        codes.append(e.code().name)
                assert time.time() - t0 < 10
    finally:
        done.set()
        th.join(timeout=5)
        py.join(timeout=5)
        srv.stop()
    # the first batch (idle dispatch: whatever had arrived) ran; everything
    # later was still waiting when the endpoint closed
    assert len(codes) == 14 and set(codes) <= {"OK", "UNAVAILABLE"}, codes
    assert 1 <= codes.count("OK") <= 4 and codes.count("UNAVAILABLE") >= 10, codes




def test_queue_drain_spreads_over_the_pool():
    """Round-5 ADVICE: more requests in flight than the slots hold park in the
    FIFO queue; the lane that frees a slot moves >= 4 of them in at once,
    which runs on the drain pool (pooled_drains counts it).  Every request is
    answered with its own rows, and the pool threads carry the process-wide
    CPU mask, not the mask of whichever (pinned) lane thread drained first."""
    import os
    srv = _C.Http2Server("127.0.0.1", 0, 2)
    ep = srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [64])], [("y", T.DT_FLOAT, [64])], 8, 5000000)
    bufs = []
    for k in range(2):
        xin, yout = np.zeros((8, 64), np.float32), np.zeros((8, 64), np.float32)
        srv.set_slot_buffers(ep, k, [xin.ctypes.data], [yout.ctypes.data])
        bufs.append((xin, yout))
    srv.set_route("m", "serving_default", -1, ep)
    stop = threading.Event()
    gate = threading.Event()

    def lane(k):
        cpu = sorted(os.sched_getaffinity(0))[0]
        os.sched_setaffinity(0, {cpu})          # a pinned lane thread, as bench.py does
        xin, yout = bufs[k]
        while not stop.is_set():
            n = srv.acquire(ep, k, 50)
            if n < 0:
                return
            if n == 0:
                continue
            gate.wait(10)                       # hold the slot until the queue has built up
            yout[:n] = xin[:n] * 3
            srv.complete(ep, k)

    ts = [threading.Thread(target=lane, args=(k,), daemon=True) for k in range(2)]
    srv.start()
    for t in ts:
        t.start()
    spec = native.spec_tuple("m", None, None, "serving_default")
    xs = [np.full((1, 64), i, np.float32) for i in range(48)]
    try:
        with grpc.insecure_channel(f"127.0.0.1:{srv.port}") as ch:
            stub = ch.unary_unary(PREDICT)
            with cf.ThreadPoolExecutor(48) as ex:
                futs = [ex.submit(stub, native.encode_predict_request(spec, {"x": x}), timeout=30) for x in xs]
                time.sleep(0.5)                 # 16 rows in the two slots, the rest queued
                gate.set()
                ys = [_y(f.result()) for f in futs]
        for x, y in zip(xs, ys):
            np.testing.assert_array_equal(y, x * 3)
        st = srv.endpoint_stats(ep)
        assert st["pooled_drains"] >= 1, st
        assert st["copy_errors"] == 0, st
        main_mask = os.sched_getaffinity(os.getpid())
        def comm(t):                            # a thread (e.g. a grpc worker) may exit mid-scan
            try:
                with open(f"/proc/self/task/{t}/comm") as f:
                    return f.read().strip()
            except FileNotFoundError:
                return None
        drains = [int(t) for t in os.listdir("/proc/self/task") if comm(t) == "tfs-drain"]
        assert len(drains) >= 3
        for tid in drains:
            assert os.sched_getaffinity(tid) == main_mask
    finally:
        stop.set()
        gate.set()
        srv.remove_endpoint(ep)
        for t in ts:
            t.join(timeout=5)
        srv.stop()
