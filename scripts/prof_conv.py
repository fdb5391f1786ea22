"""One conv layer shape, selected tile configs, many launches (for rocprofv3 --pmc).

    python scripts/prof_conv.py --shape 32,14,14,256,3,256 --cfgs 3,5,8
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="32,14,14,256,3,256", help="N,H,W,C,k,Cout")
    ap.add_argument("--cfgs", default="3")
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    n, h, w, c, k, co = (int(v) for v in a.shape.split(","))
    x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
    wt = (torch.randn(co, k * k * c, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.zeros(co, device="cuda")
    pad = k // 2
    for cfg in (int(v) for v in a.cfgs.split(",")):
        fn = lambda: hip().conv2d(x, wt, b, None, k, k, 1, 1, pad, pad, pad, pad, ACT["relu"], cfg,  # noqa
                                  splits=a.splits)
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        print(f"cfg {cfg}: {s.elapsed_time(e) / a.iters * 1e3:.1f} us")


if __name__ == "__main__":
    main()
