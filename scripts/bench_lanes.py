"""GPU-side serving ceiling: ResNet-50 HIP graphs replayed concurrently on
L lanes (one HIP stream each, as the native lane workers drive them), with and
without the per-batch H2D of the f32 request rows and D2H of the outputs.

    python scripts/bench_lanes.py --batch 32 --lanes 1 2 4
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lanes", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--iters", type=int, default=60)
    args = ap.parse_args()
    from rust_tensorflow_serving2_amd.models import resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    resnet.export(path)
    nl = max(args.lanes)
    s = Servable("resnet", 1, path, ServableOptions(device="cuda:0", max_batch_size=args.batch,
                                                    allowed_batch_sizes=(args.batch,), lanes=nl))
    r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
    b = args.batch
    lanes = r.lanes[:nl]
    for i in range(nl):
        r.lane_host_pointers(i)   # captures every bucket on the lane
    x = np.random.default_rng(0).random((b, 224, 224, 3), dtype=np.float32)
    for lane in lanes:
        lane.host_in[0][:b].copy_(torch.from_numpy(x))

    def step(lane, copies):
        with torch.cuda.stream(lane.stream):
            if copies:
                for h, d in zip(lane.host_in, lane.static_in[b]):
                    d[:b].copy_(h[:b], non_blocking=True)
            lane.graphs[b].replay()
            if copies:
                for so, ho in zip(lane.static_out[b], lane.host_out):
                    ho[:b].copy_(so[:b], non_blocking=True)

    for copies in (False, True):
        for L in args.lanes:
            use = lanes[:L]
            for _ in range(3):
                for ln in use:
                    step(ln, copies)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for i in range(args.iters):
                step(use[i % L], copies)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            print(json.dumps({"lanes": L, "copies": copies, "batch": b,
                              "img_per_s": round(args.iters * b / dt, 1),
                              "ms_per_batch": round(dt / args.iters * 1e3, 4)}), flush=True)


if __name__ == "__main__":
    main()
