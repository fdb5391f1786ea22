"""Launch one conv layer config repeatedly (a target for rocprofv3 --pmc passes).

    python scripts/one_conv.py --h 28 --cin 128 --cout 128 --k 3 --s 1 --cfg 2 --iters 50
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32)
    ap.add_argument("--h", type=int, default=28)
    ap.add_argument("--cin", type=int, default=128)
    ap.add_argument("--cout", type=int, default=128)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--s", type=int, default=1)
    ap.add_argument("--cfg", type=int, nargs="+", default=[2])
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    pad = a.k // 2
    x = torch.randn(a.n, a.h, a.h, a.cin, device="cuda").to(torch.bfloat16)
    kp = -(-a.k * a.k * a.cin // 64) * 64
    w = (torch.randn(a.cout, kp, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.zeros(a.cout, device="cuda")
    for cfg in a.cfg:
        for _ in range(a.iters):
            hip().conv2d(x, w, b, None, a.k, a.k, a.s, a.s, pad, pad, pad, pad, ACT["relu"], cfg, None, False,
                         a.splits)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
