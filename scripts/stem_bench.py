"""Time the fused ResNet stem kernel (hip().stem_pool) alone: b32 / b1
224x224x3 fp32 requests, 64 output channels, ReLU, SAME pool -- the shape of
ResNet-50's stem.  For rocprofv3 --pmc passes and quick A/B timing.

    python scripts/stem_bench.py --batch 32 --iters 50
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    x = torch.rand(a.batch, 224, 224, 3, device="cuda")
    w = (torch.randn(64, 256, device="cuda") * 0.05).to(torch.bfloat16)
    b = torch.zeros(64, device="cuda")
    run = lambda: hip().stem_pool(x, w, b, 3, 3, 3, 3, ACT["relu"], 0, 1, 0, 1)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    e1.synchronize()
    print(f"stem_pool b{a.batch}: {e0.elapsed_time(e1) * 1e3 / a.iters:.2f} us/launch (eager, back to back)")


if __name__ == "__main__":
    main()
