"""Which GPU kernels each compiled-program step launches (torch.profiler,
one eager run with a record_function range per step).  Finds stray kernels
(copies, torch elementwise / softmax) in a serving graph."""
import argparse
import os
import sys
import tempfile

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50", choices=["resnet50", "bert-base"])
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    from torch.profiler import ProfilerActivity, profile, record_function
    from rust_tensorflow_serving2_amd.models import bert, resnet
    from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions
    path = os.path.join(tempfile.mkdtemp(), "1")
    opts = ServableOptions(device="cuda:0", max_batch_size=args.batch, allowed_batch_sizes=(args.batch,))
    b = args.batch
    rng = np.random.default_rng(0)
    if args.model == "bert-base":
        bert.export(path, seed=0)
        s = Servable("bert", 1, path, opts)
        r = s.runner("serving_default", ["input_ids", "input_mask", "segment_ids"], ["pooled_output", "probabilities"])
        feeds = [torch.from_numpy(rng.integers(0, 30522, (b, 128)).astype(np.int32)).cuda(),
                 torch.ones((b, 128), dtype=torch.int32, device="cuda"),
                 torch.zeros((b, 128), dtype=torch.int32, device="cuda")]
    else:
        resnet.export(path)
        s = Servable("resnet", 1, path, opts)
        r = s.runner("serving_default", ["input"], ["classes", "probabilities"])
        feeds = [torch.rand((b, 224, 224, 3), device="cuda")]
    prog = r.program
    prog.run(feeds)                       # tune + warm
    torch.cuda.synchronize()
    steps = prog.steps

    def wrapped(i, fn):
        def call(ctx, node, ins):
            with record_function(f"step{i:03d} {node.op} {node.name}"):
                return fn(ctx, node, ins)
        return call
    prog.steps = [(wrapped(i, fn), node, a, o) for i, (fn, node, a, o) in enumerate(steps)]
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        outs = prog.run(feeds)
        r._finish(outs)
        torch.cuda.synchronize()
    prog.steps = steps
    # kernels per step: device events whose launch happened inside the step's range
    ranges = [(e.time_range.start, e.time_range.end, e.name) for e in prof.events()
              if e.name.startswith("step")]
    ranges.sort()
    kernels = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    cpu_launch = {}
    for e in prof.events():
        for k in e.kernels if hasattr(e, "kernels") else []:
            cpu_launch.setdefault(k.name, []).append(e.time_range.start)
    print(f"{len(kernels)} device events over {len(steps)} steps")
    for st, en, name in ranges:
        inside = [e for e in prof.events() if e.device_type != torch.autograd.DeviceType.CUDA and
                  st <= e.time_range.start <= en and e.name != name and not e.name.startswith("step")]
        launched = []
        for e in inside:
            for k in getattr(e, "kernels", []):
                launched.append(k.name[:70])
        print(f"{name[:80]:80s} -> {launched}")
    print("-- all device kernels (name, us)")
    for e in kernels:
        print(f"{e.name[:90]:90s} {e.time_range.elapsed_us():8.1f}")


if __name__ == "__main__":
    main()
