"""Time the in-graph host -> device row copy (`h2d_rows`) against an SDMA
hipMemcpyAsync of the same pinned bytes, one copy per graph replay / call
(median of 200).  TFSERVE_H2D_PER picks the kernel's 16-B pieces per thread.

    TFSERVE_H2D_PER=1 python scripts/h2d_probe.py --bytes 301056
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=301056)
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    host = torch.randint(0, 100, (a.bytes,), dtype=torch.uint8).pin_memory()
    dev = torch.empty(a.bytes, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        hip().h2d_rows(host, dev)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        hip().h2d_rows(host, dev)

    def timed(fn):
        ts = []
        for _ in range(a.iters):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            with torch.cuda.stream(s):
                e0.record()
                fn()
                e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(statistics.median(ts), 2)

    k_us = timed(g.replay)
    c_us = timed(lambda: dev.copy_(host, non_blocking=True))
    assert torch.equal(dev.cpu(), host)
    print(json.dumps({"bytes": a.bytes, "per": os.environ.get("TFSERVE_H2D_PER", "4"), "graph_kernel_us": k_us,
                      "sdma_copy_us": c_us}), flush=True)


if __name__ == "__main__":
    main()
