"""For every tunable launch of a model's program at one batch bucket: the
isolated (cold single-launch) time of each tile candidate next to the
whole-graph replay time with that candidate swapped in.  Shows how far the
isolated ranking is from the in-graph one (ops.graph_tune's premise).

    python scripts/probe_graph_tune.py --model bert-base --batch 32 --top 8
"""
import argparse
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base", choices=["resnet50", "bert-base"])
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("--min-ms", type=float, default=0.012)
    a = ap.parse_args()
    import torch
    from rust_tensorflow_serving2_amd import ops
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    opts = ServableOptions(device="cuda:0", max_batch_size=a.batch, allowed_batch_sizes=(a.batch,),
                           graph_autotune=False)
    rng = np.random.default_rng(0)
    if a.model == "bert-base":
        bert.export(path, seed=0)
        s = Servable("bert", 1, path, opts)
        r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"])
        x = [rng.integers(0, 30522, (a.batch, 128)).astype(np.int32), np.ones((a.batch, 128), np.int32),
             np.zeros((a.batch, 128), np.int32)]
    else:
        resnet.export(path)
        s = Servable("resnet", 1, path, opts)
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        x = [rng.random((a.batch, 224, 224, 3), dtype=np.float32)]
    lane = r.lanes[0]
    r.run(x)
    ins = lane.static_in[a.batch]
    with torch.cuda.stream(lane.stream), ops.record_tuned_keys() as keys:
        r.program.run(ins)
    lane.stream.synchronize()
    base = r._replay_ms(lane, ins)
    print(f"baseline replay {base * 1e3:.1f} us, {len(keys)} keys")
    for k, uses in sorted(keys.items(), key=lambda kv: -ops._TUNE_TIMES.get(kv[0], [(0,)])[0][0] * kv[1]):
        times = ops._TUNE_TIMES.get(k)
        if not times or times[0][0] < a.min_ms:
            continue
        cur = ops._TUNED[k]
        print(f"{k} x{uses} picked {cur}")
        for t, c in times[:a.top]:
            ops._TUNED[k] = c
            g = r._replay_ms(lane, ins)
            print(f"   cand {c}: isolated {t * 1e3:7.1f} us   graph {g * 1e3:8.1f} us ({(g - base) * 1e3:+.1f})")
        ops._TUNED[k] = cur


if __name__ == "__main__":
    main()
