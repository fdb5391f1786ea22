"""Request logging (ModelConfig.logging_config; reference
protos/tensorflow_serving/config/logging_config.proto:15,
model_server_config.proto:67): the native TFRecord writer (framing, masked
crc32c, sampling), the C++ fast path submitting sampled Predicts from its lane
threads (streamed and buffered requests logged byte-exact), and the Python
slow path writing through the same writer."""
import asyncio
import concurrent.futures as cf
import threading

import numpy as np
import pytest

from rust_tensorflow_serving2_amd import _C, native
from rust_tensorflow_serving2_amd.schema import serving
from rust_tensorflow_serving2_amd.utils import tensors as T
from rust_tensorflow_serving2_amd.utils.request_log import TFRecordWriter, read_tfrecords

import grpc

ROW = 20000
PREDICT = "/tensorflow.serving.PredictionService/Predict"


def test_native_writer_frames_and_crcs(tmp_path):
    path = str(tmp_path / "log.tfrecord")
    lg = _C.RequestLog(path, 1.0)
    rng = np.random.default_rng(0)
    recs = [rng.bytes(int(n)) for n in [0, 1, 7, 1000, 300000] + list(rng.integers(0, 5000, 60))]
    for r in recs:
        assert lg.submit_record(r)
    lg.flush()
    assert list(read_tfrecords(path)) == recs
    assert lg.stats()["written"] == len(recs) and lg.stats()["dropped"] == 0
    lg.close()
    assert not lg.submit_record(b"late")          # closed: dropped, never written
    # byte-identical to the plain Python framing
    ref = str(tmp_path / "ref.tfrecord")
    w = TFRecordWriter(ref)
    for r in recs:
        w.write(r)
    w.close()
    assert open(ref, "rb").read() == open(path, "rb").read()
    # a flipped payload byte is detected
    data = bytearray(open(path, "rb").read())
    data[12 + 3] ^= 0xFF                           # the 1st (empty) record's payload crc
    open(path, "wb").write(bytes(data))
    with pytest.raises(IOError):
        list(read_tfrecords(path))


def test_sampling_rate(tmp_path):
    for rate, lo, hi in [(0.0, 0, 0), (1.0, 40000, 40000), (0.25, 9400, 10600)]:
        lg = _C.RequestLog(str(tmp_path / f"s{rate}.tfrecord"), rate)
        n = sum(lg.sample() for _ in range(40000))
        assert lo <= n <= hi, (rate, n)
        lg.close()


def test_writer_drops_when_behind(tmp_path):
    lg = _C.RequestLog(str(tmp_path / "small.tfrecord"), 1.0, max_pending=1000)
    ok = [lg.submit_record(b"x" * 600) for _ in range(50)]
    lg.flush()
    st = lg.stats()
    assert st["written"] == sum(ok) and st["dropped"] == 50 - sum(ok) and st["written"] >= 1
    lg.close()


class _FastServer:
    """A fast-path endpoint served by a Python 'GPU lane' (y = 2x + 1)."""

    def __init__(self):
        self.srv = _C.Http2Server("127.0.0.1", 0, 2)
        self.ep = self.srv.add_endpoint("m", 1, "serving_default", [("x", T.DT_FLOAT, [ROW])],
                                        [("y", T.DT_FLOAT, [ROW])], 8, 2000)
        self.slots = []
        for k in range(2):
            xin, yout = np.zeros((8, ROW), np.float32), np.zeros((8, ROW), np.float32)
            self.srv.set_slot_buffers(self.ep, k, [xin.ctypes.data], [yout.ctypes.data])
            self.slots.append((xin, yout))
        self.srv.set_route("m", "serving_default", -1, self.ep)
        self.srv.set_route("m", "serving_default", 1, self.ep)
        self.stop = threading.Event()
        self.ts = [threading.Thread(target=self._lane, args=(k,), daemon=True) for k in range(2)]
        self.srv.start()
        for t in self.ts:
            t.start()

    def _lane(self, k):
        xin, yout = self.slots[k]
        while not self.stop.is_set():
            n = self.srv.acquire(self.ep, k, 50)
            if n < 0:
                return
            if n == 0:
                continue
            yout[:n] = xin[:n] * 2 + 1
            self.srv.complete(self.ep, k)

    def call(self, body):
        with grpc.insecure_channel(f"127.0.0.1:{self.srv.port}",
                                   options=[("grpc.max_send_message_length", 1 << 30),
                                            ("grpc.max_receive_message_length", 1 << 30)]) as ch:
            return ch.unary_unary(PREDICT)(body, timeout=60)

    def close(self):
        self.stop.set()
        self.srv.remove_endpoint(self.ep)
        for t in self.ts:
            t.join(timeout=5)
        self.srv.stop()


def test_fast_path_logs_streamed_and_buffered_byte_exact(tmp_path):
    fs = _FastServer()
    path = str(tmp_path / "fast.tfrecord")
    lg = _C.RequestLog(path, 1.0)
    fs.srv.set_endpoint_log(fs.ep, lg)
    try:
        rng = np.random.default_rng(1)
        sent = {}
        for i in range(10):
            x = rng.standard_normal((1 + i % 2, ROW)).astype(np.float32)
            filt = ["y"] if i % 3 == 2 else []     # output_filter after the inputs: buffered, not streamed
            body = native.encode_predict_request(native.spec_tuple("m", 1, None, ""), {"x": x}, output_filter=filt)
            sent[body] = fs.call(body)
        st = fs.srv.stats()
        assert st["fast_path"] == 10 and 0 < st["streamed"] < 10
        lg.flush()
        recs = [serving.PredictionLog.FromString(r) for r in read_tfrecords(path)]
        assert len(recs) == 10
        for pl in recs:
            req = pl.predict_log.request.SerializeToString()
            assert req in sent                                     # the request exactly as received
            assert pl.predict_log.response.SerializeToString() == sent[req]
            md = pl.log_metadata
            assert (md.model_spec.name, md.model_spec.version.value, md.model_spec.signature_name) == \
                ("m", 1, "serving_default")
            assert md.sampling_config.sampling_rate == 1.0 and list(md.saved_model_tags) == ["serve"]
        # logging off again: nothing more is written
        fs.srv.set_endpoint_log(fs.ep, None)
        fs.call(next(iter(sent)))
        lg.flush()
        assert len(list(read_tfrecords(path))) == 10
    finally:
        fs.close()
        lg.close()


def test_fast_path_samples_at_the_configured_rate(tmp_path):
    fs = _FastServer()
    path = str(tmp_path / "half.tfrecord")
    lg = _C.RequestLog(path, 0.5)
    fs.srv.set_endpoint_log(fs.ep, lg)
    try:
        x = np.ones((1, ROW), np.float32)
        body = native.encode_predict_request(native.spec_tuple("m", None, None, ""), {"x": x})
        with cf.ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda _: fs.call(body), range(200)))
        lg.flush()
        n = len(list(read_tfrecords(path)))
        assert 60 <= n <= 140, n
    finally:
        fs.close()
        lg.close()


def test_model_server_logging_config_slow_path(tmp_path, hpt_path):
    """CPU servable (Python core): Predict + Classify land in the model's log
    file as predict_log / classify_log records."""
    from rust_tensorflow_serving2_amd.client import TensorflowServing
    from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions
    cfg = serving.ModelServerConfig()
    mc = cfg.model_config_list.config.add(name="half_plus_two", base_path=hpt_path, model_platform="tensorflow")
    mc.logging_config.log_collector_config.filename_prefix = str(tmp_path / "hpt")
    mc.logging_config.sampling_config.sampling_rate = 1.0
    srv = ModelServer(ServerOptions(port=0, model_config=cfg)).start()
    try:
        async def go():
            c = await TensorflowServing.new().hostname("127.0.0.1").port(srv.port).build()
            for v in (1.0, 2.0, 3.0):
                await c.predict_tensors("half_plus_two", {"x": np.array([[v]], np.float32)})
            k = await TensorflowServing.new().hostname("127.0.0.1").port(srv.port) \
                .signature_name("classify_x_to_y").build()
            await k.classify("half_plus_two", {"x": [3.0]})
        asyncio.run(go())
        lg = srv.request_logs.get("half_plus_two")
        lg.flush()
        recs = [serving.PredictionLog.FromString(r) for r in read_tfrecords(lg.path)]
        kinds = [pl.WhichOneof("log_type") for pl in recs]
        assert kinds.count("predict_log") == 3 and kinds.count("classify_log") == 1
        xs = sorted(T.tensor_proto_to_numpy(pl.predict_log.request.inputs["x"]).item()
                    for pl in recs if pl.WhichOneof("log_type") == "predict_log")
        assert xs == [1.0, 2.0, 3.0]
        assert all(pl.log_metadata.model_spec.name == "half_plus_two" for pl in recs)
    finally:
        srv.stop()
