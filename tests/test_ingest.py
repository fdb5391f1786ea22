"""fp32 -> bf16 ingest on the fast path (csrc/ingest.h): the IO threads convert
an fp32 request tensor to bf16 while copying it into its batch row, for inputs
whose device program reads them as bf16 (the ResNet stem).  The conversion is
round-to-nearest-even (the device's v_cvt_pk_bf16_f32 rounding) and must be
exact for streamed payloads whose DATA frames split a float."""
import concurrent.futures as cf
import threading

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import _C, native
from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.utils import tensors as T

import grpc

ROW = 20001          # odd row length (80 KB): rows and frames split floats at odd offsets
PREDICT = "/tensorflow.serving.PredictionService/Predict"


def bf16_ref(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16 bits; NaN stays NaN, fp32 denormals
    round to bf16 denormals (the device's v_cvt_pk_bf16_f32 under HIP's default
    fp32 mode, which keeps denormals)."""
    u = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7fff + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    nan = (u & 0x7fffffff) > 0x7f800000
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


def bf16_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 1000, 4099])
def test_conversion_matches_rne_reference(n):
    rng = np.random.default_rng(n)
    x = (rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))).astype(np.float32)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.4e38, 1.0 + 2 ** -8,
                        1.0 + 3 * 2 ** -8, 255.0, 0.5], np.float32)
    x[:min(n, len(special))] = special[:min(n, len(special))]
    got = np.frombuffer(_C.ingest_f32_to_bf16(x.tobytes()), np.uint16)
    want = bf16_ref(x)
    nan = np.isnan(x)
    np.testing.assert_array_equal(got[~nan], want[~nan])
    assert np.all(np.isnan(bf16_to_f32(got[nan])))
    if n >= 10:   # ties go to even: 1 + 2^-8 -> 1.0, 1 + 3 * 2^-8 -> 1 + 2^-6
        assert bf16_to_f32(got[8:10]).tolist() == [1.0, 1.0 + 2 ** -6]


@pytest.mark.parametrize("where", [0, 5, 31, 32, 63, 64])
def test_denormals_keep_their_bits_in_every_block(where):
    """A denormal anywhere in a 32-value block (the AVX-512 path's unit, whose
    instruction reads denormals as zero) rounds exactly like the scalar path."""
    x = np.full(96, 1.5, np.float32)
    x[where] = np.float32(3e-39)
    x[(where + 7) % 96] = np.float32(-1.17e-38)
    got = np.frombuffer(_C.ingest_f32_to_bf16(x.tobytes()), np.uint16)
    np.testing.assert_array_equal(got, bf16_ref(x))
    assert got[where] != 0 and bf16_to_f32(got[where:where + 1])[0] > 0


def test_torch_agrees_on_normal_values():
    import torch
    x = np.random.default_rng(7).standard_normal(100_000).astype(np.float32)
    got = np.frombuffer(_C.ingest_f32_to_bf16(x.tobytes()), np.uint16)
    ref = torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    np.testing.assert_array_equal(got, ref)


@pytest.fixture()
def bf16_server():
    """An endpoint whose fp32 input lands in its slots as bf16 (4th spec field)."""
    srv = _C.Http2Server("127.0.0.1", 0, 2)
    ep = srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [ROW], T.DT_BFLOAT16)],
                          [("y", T.DT_FLOAT, [ROW])], 8, 3000)
    slots = []
    for k in range(2):
        xin = np.zeros((8, ROW), np.uint16)
        yout = np.zeros((8, ROW), np.float32)
        srv.set_slot_buffers(ep, k, [xin.ctypes.data], [yout.ctypes.data])
        slots.append((xin, yout))
    srv.set_route("m", "serving_default", -1, ep)
    stop = threading.Event()

    def lane(k):
        xin, yout = slots[k]
        while not stop.is_set():
            n = srv.acquire(ep, k, 50)
            if n < 0:
                return
            if n == 0:
                continue
            yout[:n] = bf16_to_f32(xin[:n]) * 2 + 1
            srv.complete(ep, k)

    ts = [threading.Thread(target=lane, args=(k,), daemon=True) for k in range(2)]
    srv.start()
    for t in ts:
        t.start()
    yield srv
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
    return T.tensor_proto_to_numpy(serving.PredictResponse.FromString(raw).outputs["y"])


def test_streamed_and_buffered_rows_are_converted(bf16_server):
    srv = bf16_server
    rng = np.random.default_rng(1)
    reqs = []
    for i in range(16):
        n = 1 + i % 3
        x = rng.standard_normal((n, ROW)).astype(np.float32)
        filt = ["y"] if i % 4 == 3 else []        # output_filter after the inputs -> buffered path
        body = native.encode_predict_request(native.spec_tuple("m", None, None, ""), {"x": x}, output_filter=filt)
        reqs.append((x, body))
    for x, body in reqs[:6]:
        np.testing.assert_array_equal(_y(_call(srv.port, body)), bf16_to_f32(bf16_ref(x)) * 2 + 1)
    st = srv.stats()
    assert st["streamed"] >= 4 and st["direct_bytes"] == 0   # converting rows never take raw recv()s
    with cf.ThreadPoolExecutor(8) as ex:
        outs = list(ex.map(lambda r: _call(srv.port, r[1]), reqs[6:]))
    for (x, _b), raw in zip(reqs[6:], outs):
        np.testing.assert_array_equal(_y(raw), bf16_to_f32(bf16_ref(x)) * 2 + 1)
    assert srv.stats()["fast_path"] == 16


def test_loadgen_streams_convert_exactly(bf16_server):
    """The native client's frames (other split points) over many streams."""
    srv = bf16_server
    xs = [np.random.default_rng(n).standard_normal((n, ROW)).astype(np.float32) for n in (1, 3, 8)]
    bodies = [native.encode_predict_request(native.spec_tuple("m", None, None, ""), {"x": x}) for x in xs]
    r = _C.run_loadgen("127.0.0.1", srv.port, PREDICT, bodies, 60, 16, 2, 2, 120.0)
    assert r["ok"] == 60 and r["errors"] == 0, r["first_error"]
    for x, body in zip(xs, bodies):
        np.testing.assert_array_equal(_y(_call(srv.port, body)), bf16_to_f32(bf16_ref(x)) * 2 + 1)


def test_unsupported_slot_dtype_is_rejected():
    srv = _C.Http2Server("127.0.0.1", 0, 1)
    with pytest.raises(ValueError):
        srv.add_endpoint("m", 1, "s", [("x", T.DT_INT32, [4], T.DT_BFLOAT16)], [("y", T.DT_FLOAT, [4])], 8, 3000)
