"""ResNet-50 b32 engine throughput with K batches in flight at once (the
serving regime: each fast-path lane replays its own HIP graph on its own
stream).  Prints per-batch ms for K = 1..lanes and the tile picks.

TFSERVE_GRAPH_TUNE_CONC=1 reproduces the isolated-replay tuner."""
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
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert-base"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--lanes", type=int, default=4)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--save-tuned", default="", help="write the tile picks (ops.save_tuned_cache format) here")
    ap.add_argument("--only-k", type=int, default=0,
                    help="time only k batches in flight (graphs only, no copies): a clean window for a "
                         "rocprofv3 kernel trace of the serving regime")
    ap.add_argument("--buckets", type=int, nargs="*", default=None,
                    help="capture these batch buckets too (all tuned; only --batch is timed)")
    args = ap.parse_args()
    from rust_tensorflow_serving2_amd import ops
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    opts = ServableOptions(device="cuda:0", max_batch_size=args.batch,
                           allowed_batch_sizes=tuple(sorted(set(args.buckets or []) | {args.batch})),
                           lanes=args.lanes)
    if args.model == "bert-base":
        bert.export(path, seed=0)
        s = Servable("bert", 1, path, opts)
        r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"])
    else:
        resnet.export(path)
        s = Servable("resnet", 1, path, opts)
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
    t0 = time.perf_counter()
    for i in r.fast_lanes():
        r.lane_host_pointers(i)
    t_cap = time.perf_counter() - t0
    b = args.batch
    lanes = [r.lanes[i] for i in r.fast_lanes()]
    res = {"model": args.model, "batch": b, "capture_s": round(t_cap, 2),
           "tune_conc": r.tune_concurrency(b)}
    if args.only_k:
        gs = [(l.graphs[b], l.stream) for l in lanes[:args.only_k]]
        for g, st in gs:
            with torch.cuda.stream(st):
                g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            for g, st in gs:
                with torch.cuda.stream(st):
                    g.replay()
        torch.cuda.synchronize()
        res[f"ms_per_batch_k{args.only_k}"] = round((time.perf_counter() - t) * 1e3 / (args.iters * args.only_k), 4)
        print(json.dumps(res), flush=True)
        return
    for k in range(1, len(lanes) + 1):
        gs = [(l.graphs[b], l.stream) for l in lanes[:k]]
        for g, st in gs:
            with torch.cuda.stream(st):
                g.replay()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t = time.perf_counter()
            for _ in range(args.iters):
                for g, st in gs:
                    with torch.cuda.stream(st):
                        g.replay()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t) * 1e3 / (args.iters * k))
        res[f"ms_per_batch_k{k}"] = round(best, 4)
    # the serving lane's full GPU-side cycle: H2D of the live rows (SDMA),
    # graph replay, D2H of the outputs -- k lanes at once
    for k in range(1, len(lanes) + 1):
        sel = lanes[:k]
        def cycle(l):
            with torch.cuda.stream(l.stream):
                for h, d in zip(l.host_in, l.static_in[b]):
                    d[:b].copy_(h[:b], non_blocking=True)
                l.graphs[b].replay()
                for so, ho in zip(l.static_out[b], l.host_out):
                    ho[:b].copy_(so[:b], non_blocking=True)
        for l in sel:
            cycle(l)
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t = time.perf_counter()
            for _ in range(args.iters):
                for l in sel:
                    cycle(l)
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t) * 1e3 / (args.iters * k))
        res[f"ms_per_batch_with_copies_k{k}"] = round(best, 4)
    # H2D alone (SDMA): bytes of one batch's inputs per lane, k lanes at once
    nbytes = sum(h[:b].numel() * h.element_size() for h in lanes[0].host_in)
    for k in range(1, len(lanes) + 1):
        sel = lanes[:k]
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            for l in sel:
                with torch.cuda.stream(l.stream):
                    for h, d in zip(l.host_in, l.static_in[b]):
                        d[:b].copy_(h[:b], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        res[f"h2d_GBps_k{k}"] = round(nbytes * args.iters * k / dt / 1e9, 2)
    picks = {}
    for key, v in ops.tuned_table().items():
        picks[repr(key)[:90]] = list(v)
    res["picks"] = picks
    if args.save_tuned:
        res["saved_tuned"] = ops.save_tuned_cache(args.save_tuned)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
