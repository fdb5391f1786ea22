"""Regenerate the committed MI355X tile-pick table (ops/tuned_mi355x.json).

The serving runtime loads that table at start-up (ops.load_tuned_cache) so a
server does not autotune its kernels on every start; picks are keyed by the
exact launch shape and only used when the table's config-table schema, gfx
arch and CU count match.  This captures every batch bucket of the served
models exactly as the runtime does (4 lanes: the largest bucket tuned for the
concurrent serving regime by the whole-graph tuner) and writes all picks.

    python scripts/make_tuned_cache.py --out rust_tensorflow_serving2_amd/ops/tuned_mi355x.json
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--models", nargs="*", default=["resnet50", "bert-base"])
    ap.add_argument("--buckets", type=int, nargs="*", default=[1, 2, 4, 8, 16, 32])
    ap.add_argument("--lanes", type=int, default=4)
    a = ap.parse_args()
    os.environ["TFSERVE_TUNED_CACHE"] = "0"         # tune from scratch
    from rust_tensorflow_serving2_amd import ops
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    opts = ServableOptions(device="cuda:0", max_batch_size=max(a.buckets), allowed_batch_sizes=tuple(a.buckets),
                           lanes=a.lanes)
    for m in a.models:
        path = os.path.join(tempfile.mkdtemp(), "1")
        t0 = time.perf_counter()
        if m == "bert-base":
            bert.export(path, seed=0)
            s = Servable("bert", 1, path, opts)
            r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"],
                         ["pooled_output", "probabilities"])
        else:
            resnet.export(path, version="v2" if m == "resnet50-v2" else "v1.5")
            s = Servable("resnet", 1, path, opts)
            r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        for i in r.fast_lanes():
            r.lane_host_pointers(i)                 # captures every bucket (tunes on the way)
        print(json.dumps({"model": m, "tune_s": round(time.perf_counter() - t0, 1),
                          "picks_so_far": len(ops.tuned_table())}), flush=True)
    n = ops.save_tuned_cache(a.out)
    print(json.dumps({"written": a.out, "picks": n}), flush=True)


if __name__ == "__main__":
    main()
