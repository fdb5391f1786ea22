"""BASELINE config 1: half_plus_two on CPU over the native HTTP/2 front end,
20,000 Predicts at 32 in flight (native load generator), per-request Python
path vs the batched C++ fast path (server/cpu_runtime.py)."""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from rust_tensorflow_serving2_amd import _C, native
from rust_tensorflow_serving2_amd.server import native_transport
from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions
from rust_tensorflow_serving2_amd.models import half_plus_two
import tempfile
d = tempfile.mkdtemp(); base = os.path.join(d, "hpt")
half_plus_two.export(os.path.join(base, "1"))
for fast in (False, True):
    native_transport.CPU_FAST_PATH = fast
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="hpt", model_base_path=base, transport="native",
                                    file_system_poll_wait_seconds=0, batch_timeout_us=500)).start()
    time.sleep(1.0)
    body = native.encode_predict_request(native.spec_tuple("hpt", None, None, ""), {"x": np.ones((1, 1), np.float32)})
    r = _C.run_loadgen("127.0.0.1", srv.port, "/tensorflow.serving.PredictionService/Predict", [body], 20000, 32, 2, 4, 120.0)
    lat = sorted(r["latency_us"]); print(json.dumps({"cpu_fast_path": fast, "ok": r["ok"], "errors": r["errors"], "rps": round(r["ok"] / r["elapsed_s"]), "p50_ms": lat[len(lat)//2] / 1e3, "p99_ms": lat[int(len(lat)*0.99)] / 1e3, "concurrency": 32}))
    srv.stop()
