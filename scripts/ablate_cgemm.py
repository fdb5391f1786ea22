"""cgemm ablations on ResNet-50 b32 conv layers: full kernel vs no operand DMA
(compute on stale LDS) vs no MFMA (DMA + epilogue only) vs neither (launch +
prologue + epilogue).  Uses the kernel's act >= 100 debug modes.

    python scripts/ablate_cgemm.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import hip  # noqa: E402


def timeit(fn, iters=20, reps=5):
    """Median over ``reps`` replays of a HIP graph holding ``iters`` launches
    (no host launch overhead in the number)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


LAYERS = [(56, 64, 64, 3, 1), (28, 128, 128, 3, 1), (14, 256, 256, 3, 1), (7, 512, 512, 3, 1), (14, 1024, 256, 1, 1)]


def main():
    n = 32
    cfgs = [int(c) for c in sys.argv[1:]] or list(range(32, 45))
    for h, cin, cout, k, s in LAYERS:
        pad = k // 2
        x = torch.randn(n, h, h, cin, device="cuda").to(torch.bfloat16)
        w = (torch.randn(cout, k * k * cin, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.zeros(cout, device="cuda")
        ho = (h + 2 * pad - k) // s + 1
        flop = 2 * n * ho * ho * cout * k * k * cin
        for cfg in cfgs:
            row = {"layer": f"{h}x{h}x{cin} k{k}->{cout}", "cfg": cfg}
            for mode, name in ((0, "full"), (101, "no_dma"), (102, "no_mma"), (103, "neither"),
                               (111, "neither_no_epi"), (116, "setup_only"), (104, "empty")):
                t = timeit(lambda: hip().conv2d(x, w, b, None, k, k, s, s, pad, pad, pad, pad, mode, cfg))
                row[name] = round(t, 1)
            row["tflops_full"] = round(flop / row["full"] / 1e6)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
