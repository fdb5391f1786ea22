"""Where a concurrency-1 Predict spends its time (bench.py's p50_c1 regime).

One ResNet-50 server (the bench's settings), one load-generator connection,
one call in flight, batch tracing on: per request, the server-side batch spans
(opened -> acquired -> H2D + graph + D2H done -> responses posted) next to the
client's round trip.  Whatever the spans do not cover is transport: the
client's send, the server's receive / decode into the slot row, and the
response's way back.

    python scripts/c1_breakdown.py [--requests 300] [--image-size 224]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=300)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--batch-timeout-us", type=int, default=2000)
    args = ap.parse_args()

    from rust_tensorflow_serving2_amd import _C, native
    from rust_tensorflow_serving2_amd.models import resnet
    from rust_tensorflow_serving2_amd.server.server import ModelServer, ServerOptions
    from rust_tensorflow_serving2_amd.server.servable import ServableOptions

    base = os.path.join(tempfile.mkdtemp(), "resnet")
    resnet.export(os.path.join(base, "1"), seed=0, image_size=args.image_size)
    so = ServableOptions(device="cuda:0", max_batch_size=args.batch, lanes=args.lanes,
                         allowed_batch_sizes=tuple(sorted({1, 2, 4, 8, 16, args.batch})))
    srv = ModelServer(ServerOptions(port=0, host="127.0.0.1", model_name="resnet", model_base_path=base,
                                    device="cuda:0", transport="native", servable=so, monitoring=False,
                                    batch_timeout_us=args.batch_timeout_us,
                                    file_system_poll_wait_seconds=0)).start()
    try:
        tr = srv.transports[0]
        for _ in range(600):
            if tr.stats().get("endpoints"):
                break
            time.sleep(0.05)
        spec = native.spec_tuple("resnet", None, None, "")
        rng = np.random.default_rng(0)
        bodies = [native.encode_predict_request(
            spec, {"input": rng.random((1, args.image_size, args.image_size, 3), dtype=np.float32)})
            for _ in range(8)]
        path = "/tensorflow.serving.PredictionService/Predict"
        lg = _C.LoadGen("127.0.0.1", srv.port, path, bodies, 1, 1, 1)
        lg.run(50, 120.0)                                 # warm-up
        native_srv = tr.srv
        native_srv.drain_trace()
        native_srv.set_tracing(True)
        r = lg.run(args.requests, 120.0)
        native_srv.set_tracing(False)
        spans = native_srv.drain_trace()
        lat = np.asarray(r["latency_us"], dtype=np.float64)
        rows = np.asarray([(acq - op, done - acq, posted - done, posted - op)
                           for _ep, _slot, _n, op, acq, _iss, done, posted in spans], dtype=np.float64)
        med = np.median(rows, axis=0) if len(rows) else [float("nan")] * 4
        out = {"requests": int(r["ok"]), "errors": int(r["errors"]), "batches": len(rows),
               "client_p50_us": round(float(np.percentile(lat, 50)), 1),
               "client_p90_us": round(float(np.percentile(lat, 90)), 1),
               "open_to_acquired_us": round(float(med[0]), 1),
               "acquired_to_gpu_done_us": round(float(med[1]), 1),
               "done_to_posted_us": round(float(med[2]), 1),
               "server_batch_span_us": round(float(med[3]), 1)}
        out["transport_and_client_us"] = round(out["client_p50_us"] - out["server_batch_span_us"], 1)
        print(json.dumps(out), flush=True)
    finally:
        srv.stop()


if __name__ == "__main__":
    main()
