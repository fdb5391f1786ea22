"""Where does a mid-size igemm launch spend its time?  Times the dense-operand
kernel at a fixed tile config while K (k-tiles per workgroup) and M (number of
workgroups) vary: the slope in K is the per-k-tile cost of one workgroup, the
intercept the fixed launch + prologue + epilogue cost.

    python scripts/probe_gemm_scaling.py --cfg 2 --n 128
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import hip  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def timeit(fn, iters=40):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, nargs="+", default=[2, 3, 0, 5, 12])
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--ms", type=int, nargs="+", default=[256 * 64, 25088, 50176])
    ap.add_argument("--ks", type=int, nargs="+", default=[64, 256, 512, 1152, 2304, 4608])
    a = ap.parse_args()
    # empty-kernel floor of this timing method
    z = torch.zeros(1, device=DEV)
    print(json.dumps({"event_floor_us": round(timeit(lambda: z.add_(1)), 2)}), flush=True)
    for cfg in a.cfg:
        for m in a.ms:
            row = {"cfg": cfg, "M": m, "N": a.n}
            for k in a.ks:
                x = torch.randn(m, k, device=DEV).to(BF)
                w = (torch.randn(a.n, k, device=DEV) * 0.05).to(BF)
                b = torch.zeros(a.n, device=DEV)
                t = timeit(lambda: hip().linear(x, w, b, None, 0, cfg, False, 1.0, None, 1))
                row[f"K{k}"] = round(t, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
