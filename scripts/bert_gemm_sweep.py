"""Graph-replay timing of every cgemm tile config on BERT-base b32's four GEMM
shapes (M = 4096): each candidate is captured as 8 back-to-back launches in a
HIP graph (the serving engine's launch mode) and timed over 20 replays.
profiles/round2/bert_gemm_sweep_deep_rings.log is this sweep with three extra
deep-ring configs (128x96 5 slots, 128x192 3 slots with 4 or 8 waves) that
were measured and dropped: none beat the existing configs on any shape.

    python scripts/bert_gemm_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, CGEMM, hip  # noqa: E402

DEV, BF = "cuda", torch.bfloat16
SHAPES = [("qkv", 4096, 2304, 768, "none", False), ("ffn1", 4096, 3072, 768, "gelu_tanh", False),
          ("ffn2", 4096, 768, 3072, "none", True), ("attn_out", 4096, 768, 768, "none", True)]


def main():
    H = hip()
    for name, m, n, k, act, has_res in SHAPES:
        x = (torch.randn(m, k, device=DEV) * 0.5).to(BF)
        w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(BF)
        b = torch.randn(n, device=DEV) * 0.1
        res = torch.randn(m, n, device=DEV).to(BF) if has_res else None
        out = torch.empty(m, n, device=DEV, dtype=BF)
        rows = []
        for cfg, (bm, bn) in sorted(CGEMM.items()):
            if bn % 64 and n % bn:
                continue
            for splits in (1, 2) if k >= 3072 else (1,):
                try:
                    H.linear(x, w, b, res, ACT[act], cfg, False, 1.0, out, splits)
                    torch.cuda.synchronize()
                except RuntimeError:
                    continue
                s = torch.cuda.Stream()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        for _ in range(8):
                            H.linear(x, w, b, res, ACT[act], cfg, False, 1.0, out, splits)
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    g.replay()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / (20 * 8)
                rows.append((us, cfg, splits, bm, bn))
                del g
        rows.sort()
        tf = 2 * m * n * k / 1e6
        print(f"== {name} M={m} N={n} K={k}: " + ", ".join(
            f"cfg {c}/{s} {bm}x{bn} {us:.1f}us ({tf / us:.0f} TF/s)" for us, c, s, bm, bn in rows[:8]), flush=True)


if __name__ == "__main__":
    main()
