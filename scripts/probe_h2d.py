"""Host->device ingest bandwidth for one ResNet-50 batch-32 input (19.3 MB fp32):

* sdma:      hipMemcpyAsync pinned -> device (copy engine), then the device-side
             ingest_c4 pass (what the serving lanes do today);
* zerocopy:  ingest_c4_from_host — the ingest kernel reads the pinned host rows
             over PCIe itself (no copy engine, no extra device pass);
each with 1 and 4 concurrent streams (the serving lanes run concurrently).
"""
import json
import time

import torch

import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import hip  # noqa: E402


def main():
    shape = (32, 224, 224, 3)
    n = 32 * 224 * 224 * 3
    L = 4
    hs = [torch.rand(shape, dtype=torch.float32).pin_memory() for _ in range(L)]
    ds = [torch.empty(shape, dtype=torch.float32, device="cuda") for _ in range(L)]
    outs = [torch.empty((32, 224, 224, 4), dtype=torch.bfloat16, device="cuda") for _ in range(L)]
    ss = [torch.cuda.Stream() for _ in range(L)]
    H = hip()
    # correctness of the zero-copy path vs the device path
    H.ingest_c4_from_host(hs[0], outs[0])
    ref = H.ingest_c4(hs[0].cuda())
    torch.cuda.synchronize()
    print(json.dumps({"zerocopy_matches": bool(torch.equal(outs[0], ref))}), flush=True)

    def sdma(i):
        ds[i].copy_(hs[i], non_blocking=True)
        H.ingest_c4(ds[i], out=outs[i])

    def zc(i):
        H.ingest_c4_from_host(hs[i], outs[i])

    for name, fn in (("sdma", sdma), ("zerocopy", zc), ("sdma_copy_only", lambda i: ds[i].copy_(hs[i], non_blocking=True))):
        for streams in (1, L):
            for _rep in range(2):
                torch.cuda.synchronize()
                t = time.perf_counter()
                iters = 20
                for _ in range(iters):
                    for i in range(streams):
                        with torch.cuda.stream(ss[i]):
                            fn(i)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t) / (iters * streams)
            print(json.dumps({"mode": name, "streams": streams, "ms_per_batch": round(dt * 1e3, 3),
                              "GBps": round(n * 4 / dt / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
