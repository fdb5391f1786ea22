"""Engine-level ResNet-50 timing on one GPU: HIP-graph replay of the fused
program per batch bucket (no transport), plus a torch/MIOpen channels-last
bf16 baseline of the same network for comparison."""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 32])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--baseline", action="store_true")
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "resnet50-v2", "bert-base"])
    ap.add_argument("--graph-tune", type=int, default=1, help="whole-graph tile re-tuning at capture (0 = off)")
    args = ap.parse_args()
    import logging
    logging.basicConfig(level=logging.INFO, format="%(name)s: %(message)s")
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    opts = ServableOptions(device="cuda:0", max_batch_size=max(args.batch), graph_autotune=bool(args.graph_tune))
    if args.model == "bert-base":
        bert.export(path, seed=0)
        s = Servable("bert", 1, path, opts)
        r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"])
        flop_per_item = 2 * 85e6 * 128 + 4 * 12 * 128 * 128 * 768   # encoder GEMMs + attention, seq 128
    else:
        resnet.export(path, version="v2" if args.model == "resnet50-v2" else "v1.5")
        s = Servable("resnet", 1, path, opts)
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        flop_per_item = 2 * 4.1e9
    res = {}
    for b in args.batch:
        rng = np.random.default_rng(0)
        if args.model == "bert-base":
            x = [rng.integers(0, 30522, (b, 128)).astype(np.int32), np.ones((b, 128), np.int32),
                 np.zeros((b, 128), np.int32)]
        else:
            x = [rng.random((b, 224, 224, 3), dtype=np.float32)]
        t0 = time.perf_counter()
        r.run(x)  # capture
        t_capture = time.perf_counter() - t0
        bucket = r._bucket(b)
        g = next(l.graphs[bucket] for l in r.lanes if bucket in l.graphs)
        torch.cuda.synchronize()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            g.replay()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.iters
        # full runner path: H2D + replay + D2H
        t = time.perf_counter()
        for _ in range(args.iters // 2):
            r.run(x)
        dt_full = (time.perf_counter() - t) / (args.iters // 2)
        res[b] = {"graph_ms": dt * 1e3, "img_per_s": b / dt, "run_ms": dt_full * 1e3,
                  "tflops": flop_per_item * b / dt / 1e12, "capture_s": round(t_capture, 2)}
        print(json.dumps({"model": args.model, "batch": b, **res[b]}), flush=True)
    if args.baseline and args.model == "resnet50":
        baseline(args)


def baseline(args):
    """Same ResNet-50 v1.5 in torch (MIOpen conv, channels_last, bf16) for reference."""
    import torch.nn as nn

    def bottleneck(cin, f, s):
        layers = nn.Sequential(nn.Conv2d(cin, f, 1, bias=True), nn.ReLU(),
                               nn.Conv2d(f, f, 3, s, 1, bias=True), nn.ReLU(),
                               nn.Conv2d(f, 4 * f, 1, bias=True))
        proj = nn.Conv2d(cin, 4 * f, 1, s, bias=True) if (s != 1 or cin != 4 * f) else None
        return layers, proj

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.stem = nn.Conv2d(3, 64, 7, 2, 3)
            self.blocks = nn.ModuleList()
            self.projs = nn.ModuleList()
            cin = 64
            for si, n in enumerate((3, 4, 6, 3)):
                for bi in range(n):
                    f = 64 * 2 ** si
                    l, p = bottleneck(cin, f, 2 if (bi == 0 and si > 0) else 1)
                    self.blocks.append(l)
                    self.projs.append(p if p is not None else nn.Identity())
                    cin = 4 * f
            self.fc = nn.Linear(2048, 1001)

        def forward(self, x):
            x = torch.relu(self.stem(x))
            x = nn.functional.max_pool2d(x, 3, 2, 1)
            for l, p in zip(self.blocks, self.projs):
                x = torch.relu(l(x) + p(x))
            return torch.softmax(self.fc(x.mean((2, 3))).float(), -1)

    net = Net().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last).eval()
    for b in args.batch:
        x = torch.rand(b, 3, 224, 224, device="cuda").to(torch.bfloat16).to(memory_format=torch.channels_last)
        with torch.no_grad():
            for _ in range(5):
                net(x)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                y = net(x)
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(args.iters):
                g.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / args.iters
        print(json.dumps({"baseline_torch_miopen": True, "batch": b, "graph_ms": dt * 1e3, "img_per_s": b / dt}),
              flush=True)


if __name__ == "__main__":
    main()
