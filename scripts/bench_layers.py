"""Per-layer reference points for the ResNet-50 b32 conv GEMMs: hipBLASLt on the
equivalent *dense* GEMM (M = N*Ho*Wo, N = Cout, K = kh*kw*Cin; im2col excluded,
so this is a lower bound for what a library conv could do) next to our tuned
implicit-GEMM conv, plus HBM / MFMA rooflines.

    python scripts/bench_layers.py [--batch 32] [--cfgs 3 5 7 ...]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, candidates, hip  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
PEAK_TF = 2500.0
HBM_TBS = 5.0


def timeit(fn, iters=20, reps=5):
    """Median over ``reps`` of the mean time of ``iters`` back-to-back launches
    (amortises the ~6 us event/launch floor of single-launch timing)."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    ts.sort()
    return ts[len(ts) // 2]


# (h, cin, cout, k, stride, residual) at batch N; ResNet-50 v1.5 distinct conv shapes
LAYERS = [
    (56, 64, 64, 1, 1, False), (56, 64, 64, 3, 1, False), (56, 64, 256, 1, 1, True), (56, 256, 64, 1, 1, False),
    (56, 256, 128, 1, 1, False), (56, 128, 128, 3, 2, False), (28, 128, 512, 1, 1, True),
    (28, 512, 128, 1, 1, False), (28, 128, 128, 3, 1, False),
    (28, 512, 256, 1, 1, False), (28, 256, 256, 3, 2, False), (14, 256, 1024, 1, 1, True),
    (14, 1024, 256, 1, 1, False), (14, 256, 256, 3, 1, False),
    (14, 1024, 512, 1, 1, False), (14, 512, 512, 3, 2, False), (7, 512, 2048, 1, 1, True),
    (7, 2048, 512, 1, 1, False), (7, 512, 512, 3, 1, False),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--no-sweep", action="store_true", help="only the library reference")
    a = ap.parse_args()
    n = a.batch
    for h, cin, cout, k, s, resid in LAYERS:
        pad = k // 2
        ho = (h + 2 * pad - k) // s + 1
        M, N, K = n * ho * ho, cout, k * k * cin
        flop = 2 * M * N * K
        bytes_min = 2 * (n * h * h * cin + M * N * (2 if resid else 1) + N * K)
        r = {"layer": f"{h}x{h}x{cin} k{k}s{s}->{cout}{' +res' if resid else ''}", "M": M, "N": N, "K": K,
             "sol_mfma_us": round(flop / PEAK_TF / 1e6, 2), "sol_hbm_us": round(bytes_min / HBM_TBS / 1e6, 2)}
        xa = torch.randn(M, K, device=DEV).to(BF)
        wb = (torch.randn(N, K, device=DEV) * 0.05).to(BF)
        r["hipblaslt_dense_us"] = round(timeit(lambda: F.linear(xa, wb)), 1)
        del xa
        if not a.no_sweep:
            x = torch.randn(n, h, h, cin, device=DEV).to(BF)
            kp = -(-K // 64) * 64
            wt = (torch.randn(cout, kp, device=DEV) * 0.05).to(BF)
            b = torch.zeros(cout, device=DEV)
            res = torch.randn(n, ho, ho, cout, device=DEV).to(BF) if resid else None
            best = {"igemm": (1e9, None), "cgemm": (1e9, None)}
            halo = k == 3 and s == 1 and cin % 64 == 0
            if halo:
                best["halo"] = (1e9, None)
            for cfg, sp in candidates(M, N, K, True, cin % 64 == 0, halo=halo):
                t = timeit(lambda: hip().conv2d(x, wt, b, res, k, k, s, s, pad, pad, pad, pad, ACT["relu"], cfg,
                                                None, False, sp))
                fam = "halo" if cfg >= 48 else "cgemm" if cfg >= 32 else "igemm"
                best[fam] = min(best[fam], (t, (cfg, sp)))
            for fam, (t, c) in best.items():
                r[f"{fam}_us"] = round(t, 1)
                r[f"{fam}_cfg"] = c
            r["ours_us"] = min(r["igemm_us"], r["cgemm_us"], r.get("halo_us", 1e9))
            xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
            wn = torch.randn(cout, cin, k, k, device=DEV).to(BF).contiguous(memory_format=torch.channels_last)
            r["miopen_us"] = round(timeit(lambda: F.conv2d(xn, wn, stride=s, padding=pad)), 1)
        r["tf_ours"] = round(flop / r.get("ours_us", 1e9) / 1e6, 0)
        r["tf_blaslt"] = round(flop / r["hipblaslt_dense_us"] / 1e6, 0)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
