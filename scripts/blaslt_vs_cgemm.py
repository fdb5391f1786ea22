"""hipBLASLt (torch._addmm_activation: bias + ReLU epilogue; torch.matmul for
the BERT shapes) vs our tuned cgemm, timed like the serving graph runs them:
captured in a HIP graph, rotating over 8 operand copies (L2-cold).  A library
anchor for comparison only: the serving path never calls the library.

    python scripts/blaslt_vs_cgemm.py                 # ResNet-50 1x1 convs
    python scripts/blaslt_vs_cgemm.py --set bert      # BERT-base b32's four GEMMs (M = 4096)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, BGEMM, candidates, hip  # noqa: E402
from scripts.conv_sweep import time_graph  # noqa: E402

BF = torch.bfloat16
SHAPES = {  # name: (M, N, K) at b32
    "s1_64_64": (100352, 64, 64), "s1_256_64": (100352, 64, 256), "s2_256_128_56": (100352, 128, 256),
    "s2_512_128": (25088, 128, 512), "s3_512_256_28": (25088, 256, 512), "s3_1024_256": (6272, 256, 1024),
    "s4_1024_512_14": (6272, 512, 1024), "s4_2048_512": (1568, 512, 2048),
    "b1_s3_1024_256": (196, 256, 1024), "b1_s4_2048_512": (49, 512, 2048),
}
BERT = {"qkv": (4096, 2304, 768), "ffn1": (4096, 3072, 768), "ffn2": (4096, 768, 3072),
        "attn_out": (4096, 768, 768)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--set", default="resnet", choices=["resnet", "bert"])
    ap.add_argument("--acts", default="", help="comma list (e.g. none,gelu_tanh): also time the best config "
                                               "with each epilogue activation")
    a = ap.parse_args()
    for name, (M, N, K) in (BERT if a.set == "bert" else SHAPES).items():
        xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(8)]
        ws = [(torch.randn(N, K, device="cuda") * 0.05).to(BF) for _ in range(8)]
        b = torch.zeros(N, device="cuda", dtype=BF)
        bf = torch.zeros(N, device="cuda")
        outs = [torch.empty(M, N, device="cuda", dtype=BF) for _ in range(8)]
        if a.set == "bert":
            t_lt = time_graph(lambda i: torch.matmul(xs[i % 8], ws[i % 8].t(), out=outs[i % 8]))
        else:
            t_lt = time_graph(lambda i: torch._addmm_activation(b, xs[i % 8], ws[i % 8].t(), use_gelu=False))
        best = (1e9, None)
        big = (1e9, None)          # the big-tile ping-pong builds (kernels/bgemm.hip) apart
        for cfg, sp in candidates(M, N, K, True, True):
            try:
                t = time_graph(lambda i, cfg=cfg, sp=sp: hip().linear(xs[i % 8], ws[i % 8], bf, None, ACT["relu"], cfg,
                                                                       False, 1.0, outs[i % 8], sp))
            except RuntimeError:
                continue
            if cfg in BGEMM:
                big = min(big, (t, (cfg, sp)))
            else:
                best = min(best, (t, (cfg, sp)))
        tf = 2 * M * N * K / 1e6
        by_act = {}
        for act in filter(None, a.acts.split(",")):
            cfg, sp = best[1]
            by_act[act] = round(time_graph(lambda i: hip().linear(xs[i % 8], ws[i % 8], bf, None, ACT[act], cfg,
                                                                  False, 1.0, outs[i % 8], sp)), 2)
        print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_lt, 2),
                          "hipblaslt_tflops": round(tf / t_lt), "cgemm_us": round(best[0], 2),
                          "cgemm_tflops": round(tf / best[0]), "cgemm_cfg": best[1], "cgemm_us_by_act": by_act,
                          "bgemm_us": round(big[0], 2), "bgemm_tflops": round(tf / big[0]) if big[1] else None,
                          "bgemm_cfg": big[1]}),
              flush=True)


if __name__ == "__main__":
    main()
