"""Run one dense GEMM config repeatedly (a target for rocprofv3 --pmc passes):

    python scripts/gemm_one.py --shape 4096x3072x768 --cfg 140 --splits 1 --iters 20

Operands rotate over 8 copies (L2-cold, as scripts/blaslt_vs_cgemm.py);
prints the mean event-timed microseconds per launch."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x3072x768")
    ap.add_argument("--cfg", type=int, default=140)
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--act", default="none")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    M, N, K = (int(v) for v in a.shape.split("x"))
    xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(8)]
    ws = [(torch.randn(N, K, device="cuda") * 0.05).to(BF) for _ in range(8)]
    outs = [torch.empty(M, N, device="cuda", dtype=BF) for _ in range(8)]
    b = torch.zeros(N, device="cuda")
    run = lambda i: hip().linear(xs[i % 8], ws[i % 8], b, None, ACT[a.act], a.cfg, False, 1.0, outs[i % 8], a.splits)
    for i in range(3):
        run(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(a.iters):
        run(i)
    e1.record()
    e1.synchronize()
    print(f"{a.shape} cfg {a.cfg} splits {a.splits}: {e0.elapsed_time(e1) * 1e3 / a.iters:.2f} us/launch "
          f"({2 * M * N * K / (e0.elapsed_time(e1) * 1e-3 / a.iters) / 1e12:.0f} TF/s)")


if __name__ == "__main__":
    main()
