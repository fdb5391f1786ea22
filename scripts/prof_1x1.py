"""Memory-bound 1x1-conv probe: our igemm configs vs pure fill/copy kernels of
the same byte volume (ResNet-50 stage-2 expand: 32x56x56x64 -> 256)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402


def timeit(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    dev = "cuda"
    x = torch.randn(32, 56, 56, 64, device=dev).to(torch.bfloat16)
    w = (torch.randn(256, 64, device=dev) * 0.1).to(torch.bfloat16)
    b = torch.zeros(256, device=dev)
    res = torch.randn(32, 56, 56, 256, device=dev).to(torch.bfloat16)
    out = torch.empty(32, 56, 56, 256, device=dev, dtype=torch.bfloat16)
    big = torch.empty_like(out)
    for cfg in range(8):
        for r in (None, res):
            try:
                t = timeit(lambda: hip().conv2d(x, w, b, r, 1, 1, 1, 1, 0, 0, 0, 0, ACT["relu"], cfg, out=out))
            except RuntimeError as e:
                print(f"cfg {cfg}: {e}")
                continue
            print(f"conv1x1 cfg={cfg} residual={r is not None}: {t:.1f} us")
    print(f"fill 51MB: {timeit(lambda: out.fill_(1.0)):.1f} us")
    print(f"copy 51MB: {timeit(lambda: big.copy_(out)):.1f} us")
    print(f"add 3x51MB: {timeit(lambda: torch.add(res, big, out=out)):.1f} us")


if __name__ == "__main__":
    main()
