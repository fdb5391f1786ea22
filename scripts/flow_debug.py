"""Find the first step where the flow launch and the per-layer kernels
disagree: flow blocks built from the first k member ops of the ResNet-50 block."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.graph import flow, ops as O  # noqa: E402
from rust_tensorflow_serving2_amd.models import resnet  # noqa: E402
from rust_tensorflow_serving2_amd.server.servable import Servable, ServableOptions  # noqa: E402

base = tempfile.mkdtemp()
resnet.export(os.path.join(base, "1"), seed=0)
s = Servable("resnet", 1, os.path.join(base, "1"), ServableOptions(device="cuda:0", max_batch_size=4))
prog = s.runner("serving_default", ["input"], ["classes", "probabilities"]).program
(blk,) = [n.attrs["_impl"] for _f, n, _i, _o in prog.steps if n.op == "_FlowBlock"]
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = (torch.rand(batch, 56, 56, 64, device="cuda") * 2).to(torch.bfloat16)
ctx = O.Ctx(torch.device("cuda:0"))
for k in range(1, len(blk.subs) + 1):
    sub = flow.FlowBlock(blk.subs[:k], blk.subs[k - 1][3][-1], "dbg")
    tab = sub.table_for(x)
    ctrl = torch.zeros(tab["ctrl_ints"] + 64, dtype=torch.int32, device="cuda")
    y = sub.run_flow(x, ctrl=ctrl)
    ref = sub.run_sequential(ctx, x)
    torch.cuda.synchronize()
    rel = float((y.float() - ref.float()).norm() / ref.float().norm())
    st = tab["steps"][-1]
    print(f"k={k} op={blk.subs[k-1][1].op} mode={st['mode']} M={st['M']} N={st['N']} K={st['K']} "
          f"splits={st['splits']} err_flag={int(ctrl[2])} rel={rel:.4g}", flush=True)
    if rel > 0.02:
        d = (y.float() - ref.float()).abs().reshape(-1, st["N"])
        rows = torch.nonzero(d.amax(1) > 0.05 * ref.float().abs().max()).flatten()
        cols = torch.nonzero(d.amax(0) > 0.05 * ref.float().abs().max()).flatten()
        print("  bad rows", rows[:20].tolist(), "of", d.shape[0], " bad cols", cols[:20].tolist(), len(cols))
        break
