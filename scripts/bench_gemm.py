"""Microbenchmark of the implicit-GEMM kernel: every (tile config, split-K)
candidate on ResNet-50 b32 layer shapes + a square GEMM, vs torch (hipBLASLt /
MIOpen) on the same bf16 data.  Prints TFLOP/s per candidate."""
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, candidates, hip  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3   # us


def conv_case(n, h, w, cin, cout, k, s, pad):
    x = torch.randn(n, h, w, cin, device=DEV).to(BF)
    kp = -(-k * k * cin // 64) * 64
    wt = (torch.randn(cout, kp, device=DEV) * 0.05).to(BF)
    b = torch.zeros(cout, device=DEV)
    ho = (h + 2 * pad - k) // s + 1
    M, N, K = n * ho * ho, cout, k * k * cin
    flop = 2 * M * N * K
    res = {"shape": f"conv {n}x{h}x{w}x{cin} k{k}s{s} -> {cout}", "M": M, "N": N, "K": K}
    best = (1e9, None)
    for cfg, sp in candidates(M, N, K, True, cin % 64 == 0):
        t = timeit(lambda: hip().conv2d(x, wt, b, None, k, k, s, s, pad, pad, pad, pad, ACT["relu"], cfg,
                                        None, False, sp))
        res[f"c{cfg}s{sp}"] = round(t, 1)
        best = min(best, (t, (cfg, sp)))
    res["best_us"] = round(best[0], 1)
    res["best"] = best[1]
    res["best_tflops"] = round(flop / best[0] / 1e6, 1)
    xn = x.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wn = torch.randn(cout, cin, k, k, device=DEV).to(BF).contiguous(memory_format=torch.channels_last)
    res["torch_us"] = round(timeit(lambda: F.conv2d(xn, wn, stride=s, padding=pad)), 1)
    return res


def gemm_case(m, n, k):
    x = torch.randn(m, k, device=DEV).to(BF)
    w = (torch.randn(n, k, device=DEV) * 0.05).to(BF)
    b = torch.zeros(n, device=DEV)
    flop = 2 * m * n * k
    res = {"shape": f"gemm {m}x{n}x{k}", "M": m, "N": n, "K": k}
    best = (1e9, None)
    for cfg, sp in candidates(m, n, k, True, k % 64 == 0):
        t = timeit(lambda: hip().linear(x, w, b, None, 0, cfg, n % 8 != 0, 1.0, None, sp))
        res[f"c{cfg}s{sp}"] = round(t, 1)
        best = min(best, (t, (cfg, sp)))
    res["best_us"] = round(best[0], 1)
    res["best"] = best[1]
    res["best_tflops"] = round(flop / best[0] / 1e6, 1)
    bb = b.to(BF)
    res["torch_us"] = round(timeit(lambda: F.linear(x, w, bb)), 1)
    res["torch_tflops"] = round(flop / res["torch_us"] / 1e6, 1)
    return res


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--gemm-only":
        for c in (gemm_case(4096, 4096, 4096), gemm_case(4096, 3072, 768), gemm_case(4096, 2304, 768),
                  gemm_case(4096, 768, 3072), gemm_case(4096, 768, 768)):
            print(json.dumps(c), flush=True)
        return
    cases = [
        conv_case(32, 56, 56, 64, 64, 3, 1, 1),
        conv_case(32, 56, 56, 64, 256, 1, 1, 0),
        conv_case(32, 28, 28, 128, 128, 3, 1, 1),
        conv_case(32, 14, 14, 256, 256, 3, 1, 1),
        conv_case(32, 7, 7, 512, 512, 3, 1, 1),
        conv_case(32, 7, 7, 512, 2048, 1, 1, 0),
        gemm_case(32, 1001, 2048),
        gemm_case(4096, 4096, 4096),
        gemm_case(4096, 3072, 768),      # BERT-base b32 FFN1
        gemm_case(4096, 2304, 768),      # fused QKV
        gemm_case(4096, 768, 3072),      # FFN2
        gemm_case(4096, 768, 768),       # attention output projection
    ]
    for c in cases:
        print(json.dumps(c), flush=True)


if __name__ == "__main__":
    main()
