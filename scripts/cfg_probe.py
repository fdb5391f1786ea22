"""Time chosen cgemm tile configs on one GEMM shape (HIP-graph replay,
8 rotating L2-cold operand copies, like `blaslt_vs_cgemm.py`), or, with
`--pmc-launches N`, just run each config N times eagerly so a
`rocprofv3 --pmc` pass attributes counters per config (kernel names carry the
tile).  Comparison tool for the 16x16x32 vs 32x32x16 builds of one tile.

    python scripts/cfg_probe.py --mnk 4096,3072,768 --act gelu_tanh --cfgs 72,123
    rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT ... -- python scripts/cfg_probe.py ... --pmc-launches 20
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402
from scripts.conv_sweep import time_graph  # noqa: E402

BF = torch.bfloat16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mnk", default="4096,3072,768")
    ap.add_argument("--act", default="none", choices=sorted(ACT))
    ap.add_argument("--cfgs", default="72,123")
    ap.add_argument("--splits", type=int, default=1)
    ap.add_argument("--pmc-launches", type=int, default=0)
    a = ap.parse_args()
    M, N, K = (int(v) for v in a.mnk.split(","))
    xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(8)]
    ws = [(torch.randn(N, K, device="cuda") / K ** 0.5).to(BF) for _ in range(8)]
    bias = torch.zeros(N, device="cuda")
    outs = [torch.empty(M, N, device="cuda", dtype=BF) for _ in range(8)]
    H = hip()
    tf = 2 * M * N * K / 1e6
    for cfg in (int(c) for c in a.cfgs.split(",")):
        def run(i, cfg=cfg):
            H.linear(xs[i % 8], ws[i % 8], bias, None, ACT[a.act], cfg, False, 1.0, outs[i % 8], a.splits)
        if a.pmc_launches:
            for i in range(a.pmc_launches):
                run(i)
            torch.cuda.synchronize()
            print(json.dumps({"cfg": cfg, "launches": a.pmc_launches}), flush=True)
            continue
        us = time_graph(run)
        print(json.dumps({"mnk": [M, N, K], "act": a.act, "cfg": cfg, "splits": a.splits, "us": round(us, 2),
                          "tflops": round(tf / us)}), flush=True)


if __name__ == "__main__":
    main()
