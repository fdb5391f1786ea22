"""Per-kernel cost of the deferred-LayerNorm epilogue (hip().linear_lnx) on
BERT-base's four GEMM shapes: the plain GEMM (hip().linear), the GEMM reading
a pre-LayerNorm A (a_st, gamma folded into the weights), and the GEMM
normalising a pre-LayerNorm residual and emitting its own row partials
(r_st + stats) -- HIP-graph replays of 20 launches rotating over 4 operand
copies, median of 5.

    python scripts/lnx_probe.py [--cfgs 72 123 100 47 45]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402

BF = torch.bfloat16
SHAPES = {  # name: (M, N, K, act, residual)
    "qkv": (4096, 2304, 768, "none", False),
    "attn_out": (4096, 768, 768, "none", True),
    "ffn1": (4096, 3072, 768, "gelu_tanh", False),
    "ffn2": (4096, 768, 3072, "none", True),
}


def timed(fn, reps=20, trials=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for i in range(3):
            fn(i)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(reps):
            fn(i)
    out = []
    for _ in range(trials):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", type=int, nargs="*", default=[72, 123, 100, 47, 45, 36])
    a = ap.parse_args()
    H = hip()
    nc = 4
    for name, (M, N, K, act, resid) in SHAPES.items():
        xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(nc)]
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).to(BF) for _ in range(nc)]
        rs = [torch.randn(M, N, device="cuda").to(BF) for _ in range(nc)] if resid else [None] * nc
        b = torch.zeros(N, device="cuda")
        ast = torch.rand(M, 6, 2, device="cuda") + 1
        cs = torch.randn(N, device="cuda")
        g1, b1 = torch.ones(N, device="cuda"), torch.zeros(N, device="cuda")
        out = torch.empty(M, N, device="cuda", dtype=BF)
        row = {"shape": name, "M": M, "N": N, "K": K}
        for cfg in a.cfgs:
            res = {}
            try:
                res["plain"] = round(timed(lambda i: H.linear(xs[i % nc], ws[i % nc], b, rs[i % nc], ACT[act], cfg,
                                                              False, 1.0, out, 1)), 2)
                if resid:
                    res["r_st+stats"] = round(timed(lambda i: H.linear_lnx(
                        xs[i % nc], ws[i % nc], b, rs[i % nc], ACT[act], cfg, False, out, r_st=ast, r_gamma=g1,
                        r_beta=b1, stats=True)), 2)
                    res["stats"] = round(timed(lambda i: H.linear_lnx(
                        xs[i % nc], ws[i % nc], b, rs[i % nc], ACT[act], cfg, False, out, stats=True)), 2)
                else:
                    res["a_st"] = round(timed(lambda i: H.linear_lnx(
                        xs[i % nc], ws[i % nc], b, None, ACT[act], cfg, False, out, a_st=ast, a_colsum=cs)), 2)
            except RuntimeError as e:
                res["error"] = str(e)[:60]
            row[cfg] = res
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
