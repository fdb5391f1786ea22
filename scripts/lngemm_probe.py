"""GEMM + residual + LayerNorm: the fused kernel (hip().linear_ln, kernels/lngemm.hip)
against the two launches it replaces (the best tuned cgemm tile + layernorm),
graph-captured and rotating over 8 operand copies as scripts/conv_sweep.py.

    python scripts/lngemm_probe.py                       # BERT-base b32 attention output (4096 x 768 x 768)
    python scripts/lngemm_probe.py --shapes 4096x768x3072 128x768x768
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import candidates, hip  # noqa: E402
from scripts.conv_sweep import time_graph  # noqa: E402
from rust_tensorflow_serving2_amd.graph.fused import ln_weight_frags  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["4096x768x768", "4096x768x3072", "128x768x768"])
    a = ap.parse_args()
    H = hip()
    for shp in a.shapes:
        M, N, K = (int(v) for v in shp.split("x"))
        xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(8)]
        ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).to(BF) for _ in range(8)]
        wf = [ln_weight_frags(w) for w in ws]
        rs = [torch.randn(M, N, device="cuda").to(BF) for _ in range(8)]
        outs = [torch.empty(M, N, device="cuda", dtype=BF) for _ in range(8)]
        b, gm, bt = (torch.randn(N, device="cuda") for _ in range(3))
        res = {"shape": shp}
        for bm in (16, 32, 64):
            if H.linear_ln_supported(M, N, K, bm):
                res[f"fused_bm{bm}_us"] = round(time_graph(
                    lambda i, bm=bm: H.linear_ln(xs[i % 8], wf[i % 8], b, rs[i % 8], gm, bt, 1e-12, bm,
                                                 outs[i % 8])), 2)
        best = None
        for cfg, sp in candidates(M, N, K, True, K % 64 == 0):
            try:
                t = time_graph(lambda i: H.linear(xs[i % 8], ws[i % 8], b, rs[i % 8], 0, cfg, False, 1.0,
                                                  outs[i % 8], sp))
            except RuntimeError:
                continue
            if best is None or t < best[0]:
                best = (t, cfg, sp)
        tln = time_graph(lambda i: H.layernorm(outs[i % 8], None, gm, bt, 1e-12, rs[(i + 3) % 8]))
        res.update({"gemm_us": round(best[0], 2), "gemm_cfg": best[1:], "layernorm_us": round(tln, 2),
                    "split_us": round(best[0] + tln, 2)})
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
