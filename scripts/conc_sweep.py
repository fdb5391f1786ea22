"""Tile configs of ResNet-50 layers, isolated vs under concurrency.

The serving runtime keeps 3-4 batches in flight on separate HIP streams, so a
layer's kernels share the GPU with other batches' kernels (0.54 ms per b32
batch at 3 in flight vs 0.78 ms for one isolated replay).  A tile config that
loses in isolation because it leaves CUs idle (few, large tiles) can win there:
its idle CUs run the other streams' work.  This probe times every candidate
two ways, both as HIP-graph replays rotating over 8 operand copies (operands
in the Infinity Cache, not L2):

* ``iso``: 16 launches back to back on one stream (us per launch);
* ``conc``: ``--streams`` graphs of 16 launches each, replayed concurrently
  on their own streams (us per launch of the combined throughput).

    python scripts/conc_sweep.py                       # ResNet-50 b32 layers
    python scripts/conc_sweep.py --layers s3_1x1_in --streams 3 --top 8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, candidates, hip  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conv_sweep import LAYERS  # noqa: E402

BF = torch.bfloat16


def _graph(fn, stream, reps):
    with torch.cuda.stream(stream):
        for i in range(2):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for i in range(reps):
            fn(i)
    return g


def time_iso_conc(fns, reps=16, trials=5):
    """fns[s](i): launch i of stream s's copy.  Returns (iso us, conc us) per launch."""
    streams = [torch.cuda.Stream() for _ in fns]
    graphs = [_graph(f, st, reps) for f, st in zip(fns, streams)]
    for g in graphs:
        g.replay()
    torch.cuda.synchronize()
    iso, conc = [], []
    for _ in range(trials):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(streams[0])
        with torch.cuda.stream(streams[0]):
            graphs[0].replay()
        e1.record(streams[0])
        e1.synchronize()
        iso.append(e0.elapsed_time(e1) * 1e3 / reps)
        # concurrent: every stream waits for a start event, replays, the main stream joins
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        cur = torch.cuda.current_stream()
        start.record(cur)
        for st, g in zip(streams, graphs):
            st.wait_event(start)
            with torch.cuda.stream(st):
                g.replay()
        for st in streams:
            cur.wait_stream(st)
        end = torch.cuda.Event(enable_timing=True)
        end.record(cur)
        end.synchronize()
        conc.append(start.elapsed_time(end) * 1e3 / (reps * len(graphs)))
    iso.sort()
    conc.sort()
    return iso[len(iso) // 2], conc[len(conc) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", nargs="*", default=list(LAYERS))
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--top", type=int, default=6)
    ap.add_argument("--splits", action="store_true", help="also split-K candidates")
    ap.add_argument("--cfgs", type=int, nargs="*", default=None, help="only these tile configs")
    a = ap.parse_args()
    n = a.batch
    for name in a.layers:
        h, cin, cout, k, s, resid = LAYERS[name]
        pad = k // 2
        ho = (h + 2 * pad - k) // s + 1
        M, N, K = n * ho * ho, cout, k * k * cin
        kp = -(-K // 64) * 64
        ncopy = 8
        xs = [torch.randn(n, h, h, cin, device="cuda").to(BF) for _ in range(ncopy)]
        ws = [(torch.randn(cout, kp, device="cuda") * 0.05).to(BF) for _ in range(ncopy)]
        rs = [torch.randn(n, ho, ho, cout, device="cuda").to(BF) for _ in range(ncopy)] if resid else [None] * ncopy
        outs = [[torch.empty(n, ho, ho, cout, device="cuda", dtype=BF) for _ in range(ncopy)]
                for _ in range(a.streams)]
        b = torch.zeros(cout, device="cuda")
        halo = k == 3 and s == 1 and cin % 64 == 0
        res = []
        for cfg, sp in candidates(M, N, K, True, cin % 64 == 0, halo=halo):
            if (sp > 1 and not a.splits) or (a.cfgs and cfg not in a.cfgs):
                continue
            fns = []
            for si in range(a.streams):
                def fn(i, cfg=cfg, sp=sp, si=si):
                    j = (i + 3 * si) % ncopy
                    hip().conv2d(xs[j], ws[j], b, rs[j], k, k, s, s, pad, pad, pad, pad, ACT["relu"], cfg,
                                 outs[si][j], False, sp)
                fns.append(fn)
            try:
                ti, tc = time_iso_conc(fns)
                res.append((tc, ti, cfg, sp))
            except RuntimeError as e:
                print(f"  {name} cfg {cfg} x{sp}: {str(e)[:80]}", flush=True)
        flop = 2 * M * N * K
        by_iso = sorted(res, key=lambda r: r[1])
        by_conc = sorted(res)
        print(json.dumps({"layer": name, "M": M, "N": N, "K": K,
                          "best_iso": [(round(ti, 2), round(tc, 2), c, sp) for tc, ti, c, sp in by_iso[:a.top]],
                          "best_conc": [(round(tc, 2), round(ti, 2), c, sp) for tc, ti, c, sp in by_conc[:a.top]],
                          "tflops_iso": round(flop / by_iso[0][1] / 1e6) if res else None,
                          "tflops_conc": round(flop / by_conc[0][0] / 1e6) if res else None}), flush=True)


if __name__ == "__main__":
    main()
