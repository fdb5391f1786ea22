"""Per-kernel cost of a dependent chain of tiny kernels inside one HIP graph
(the batch-1 forward is ~55 such launches): 200 x a 1-element add captured in
a graph, replayed 20 times.  Run under different HIP runtime settings to see
what the floor depends on.

    python scripts/launch_floor.py
"""
import os

import torch


def main():
    x = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        x.add_(1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(200):
                x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / (20 * 200))
    env = {k: v for k, v in os.environ.items() if k.startswith(("HIP_", "DEBUG_CLR", "GPU_", "HSA_", "AMD_"))
           and k not in ("HSA_ENABLE_IPC_MODE_LEGACY",)}
    print(f"graph chain of tiny kernels: {best:.2f} us per kernel  env={env}", flush=True)


if __name__ == "__main__":
    main()
