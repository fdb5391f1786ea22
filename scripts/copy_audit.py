"""List the device copies (aten copy_ / clone / _to_copy) one eager run of a
served program issues, with the Python frame that asked for each: the
`__amd_rocclr_copyBuffer` / copy kernels in a replay table come from these.

    python scripts/copy_audit.py --model bert-base --batch 32
"""
import argparse
import os
import sys
import tempfile
import traceback

import numpy as np
import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

WATCH = ("aten.copy_", "aten.clone", "aten._to_copy", "aten.contiguous", "aten.index", "aten.cat")


class Audit(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = []

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func.overloadpacket)
        name = "aten." + name.split(".")[-1] if not name.startswith("aten.") else name
        if any(name.startswith(w) for w in WATCH):
            shapes = [tuple(a.shape) for a in args if isinstance(a, torch.Tensor)]
            devs = [str(a.device) for a in args if isinstance(a, torch.Tensor)]
            frames = [f for f in traceback.extract_stack()[:-1] if "rust_tensorflow_serving2_amd" in f.filename]
            where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in frames[-3:])
            self.rows.append((name, shapes, devs, where))
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bert-base")
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    from rust_tensorflow_serving2_amd.models import bert
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    bert.export(path, seed=0)
    s = Servable("bert", 1, path, ServableOptions(device="cuda:0", max_batch_size=a.batch))
    r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"])
    rng = np.random.default_rng(0)
    x = [rng.integers(0, 30522, (a.batch, 128)).astype(np.int32), np.ones((a.batch, 128), np.int32),
         np.zeros((a.batch, 128), np.int32)]
    r.run(x)
    lane = r.lanes[0]
    ins = [t[:a.batch] for t in lane.dev_in]
    with torch.cuda.device(0):
        r.program.run(ins)
        torch.cuda.synchronize()
        with Audit() as au:
            r._finish(r.program.run(ins))
        torch.cuda.synchronize()
    for name, shapes, devs, where in au.rows:
        print(f"{name:16s} {shapes} {devs} {where}")
    print(f"{len(au.rows)} copy-like ops")


if __name__ == "__main__":
    main()
