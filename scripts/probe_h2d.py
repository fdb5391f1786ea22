"""H2D bandwidth probe: pinned host -> device copies of one ResNet-50 batch-32
input (19.3 MB fp32), single stream and 3 concurrent streams."""
import time

import torch


def main():
    n = 32 * 224 * 224 * 3
    hs = [torch.empty(n, dtype=torch.float32, pin_memory=True) for _ in range(3)]
    ds = [torch.empty(n, dtype=torch.float32, device="cuda") for _ in range(3)]
    ss = [torch.cuda.Stream() for _ in range(3)]
    print("is_pinned", hs[0].is_pinned())
    for rep in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            ds[0].copy_(hs[0], non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 20
        print(f"1 stream: {dt*1e3:.3f} ms/batch  {n*4/dt/1e9:.1f} GB/s")
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(20):
            for h, d, s in zip(hs, ds, ss):
                with torch.cuda.stream(s):
                    d.copy_(h, non_blocking=True)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / 60
        print(f"3 streams: {dt*1e3:.3f} ms/batch  {n*4/dt/1e9:.1f} GB/s")
    # bf16 half-size
    hb = torch.empty(n, dtype=torch.bfloat16, pin_memory=True)
    db = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        db.copy_(hb, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 20
    print(f"bf16 1 stream: {dt*1e3:.3f} ms/batch  {n*2/dt/1e9:.1f} GB/s")


if __name__ == "__main__":
    main()
