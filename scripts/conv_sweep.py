"""Every tile config x split-K of a conv layer, timed the way the serving graph
runs it: launches captured in a HIP graph (no host overhead), rotating over 8
input / weight copies so each launch finds its operands in the Infinity Cache
but not in L2 (what a layer sees after its producer ran).

    python scripts/conv_sweep.py                 # ResNet-50 b32 stage 2-4 layers
    python scripts/conv_sweep.py --batch 1 --top 3
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, candidates, hip  # noqa: E402

BF = torch.bfloat16
LAYERS = {
    "s1_3x3": (56, 64, 64, 3, 1, False), "s2_3x3s2": (56, 128, 128, 3, 2, False), "s2_3x3": (28, 128, 128, 3, 1, False),
    "s3_3x3s2": (28, 256, 256, 3, 2, False), "s3_3x3": (14, 256, 256, 3, 1, False),
    "s4_3x3s2": (14, 512, 512, 3, 2, False), "s4_3x3": (7, 512, 512, 3, 1, False),
    "s1_1x1_in": (56, 256, 64, 1, 1, False), "s1_1x1_out": (56, 64, 256, 1, 1, True),
    "s2_1x1_in": (28, 512, 128, 1, 1, False), "s2_1x1_out": (28, 128, 512, 1, 1, True),
    "s3_1x1_in": (14, 1024, 256, 1, 1, False), "s3_1x1_out": (14, 256, 1024, 1, 1, True),
    "s4_1x1_in": (7, 2048, 512, 1, 1, False), "s4_1x1_out": (7, 512, 2048, 1, 1, True),
}


def time_graph(fn, reps=16, trials=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for i in range(2):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            fn(i)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(trials):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", nargs="*", default=list(LAYERS))
    ap.add_argument("--top", type=int, default=5)
    a = ap.parse_args()
    n = a.batch
    for name in a.layers:
        h, cin, cout, k, s, resid = LAYERS[name]
        pad = k // 2
        ho = (h + 2 * pad - k) // s + 1
        M, N, K = n * ho * ho, cout, k * k * cin
        kp = -(-K // 64) * 64
        xs = [torch.randn(n, h, h, cin, device="cuda").to(BF) for _ in range(8)]
        ws = [(torch.randn(cout, kp, device="cuda") * 0.05).to(BF) for _ in range(8)]
        rs = [torch.randn(n, ho, ho, cout, device="cuda").to(BF) for _ in range(8)] if resid else [None] * 8
        outs = [torch.empty(n, ho, ho, cout, device="cuda", dtype=BF) for _ in range(8)]
        b = torch.zeros(cout, device="cuda")
        halo = k == 3 and s == 1 and cin % 64 == 0
        res = []
        for cfg, sp in candidates(M, N, K, True, cin % 64 == 0, halo=halo):
            def fn(i, cfg=cfg, sp=sp):
                j = i % 8
                hip().conv2d(xs[j], ws[j], b, rs[j], k, k, s, s, pad, pad, pad, pad, ACT["relu"], cfg, outs[j],
                             False, sp)
            try:
                res.append((time_graph(fn), cfg, sp))
            except RuntimeError as e:
                if "launch failed" not in str(e):       # (operand modes a config does not take: silent)
                    print(f"  {name} cfg {cfg} x{sp}: {str(e)[:80]}", flush=True)
        res.sort()
        flop = 2 * M * N * K
        print(json.dumps({"layer": name, "M": M, "N": N, "K": K, "sol_mfma_us": round(flop / 2.5e9, 2),
                          "best": [(round(t, 2), c, sp) for t, c, sp in res[:a.top]],
                          "tflops": round(flop / res[0][0] / 1e6)}), flush=True)


if __name__ == "__main__":
    main()
