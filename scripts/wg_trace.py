"""Where a conv / GEMM launch spends its time, per workgroup: every workgroup
stamps the steady wall clock (100 MHz) at entry, when its first operand tile
has landed (after the first wait + barrier), after its K loop and at exit
(kernels/gemm_common.h trace_stamp; the trace buffer is set through
``hip().set_wg_trace``).  Printed per layer x config: the launch's span, how
the workgroup start times spread over it (one wave of workgroups or several),
and the median / p90 of each phase.

    python scripts/wg_trace.py --layers s1_3x3 s3_3x3 s3_1x1_in --cfgs 48:1 51:1 42:1

Operands rotate over 8 copies (as scripts/conv_sweep.py): the traced launch
finds its input in the Infinity Cache, not in L2 -- what a layer sees in the
serving graph after its producer ran.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rust_tensorflow_serving2_amd.ops import ACT, hip  # noqa: E402
from conv_sweep import LAYERS  # noqa: E402

BF = torch.bfloat16
TICK_US = 0.01      # 100 MHz steady counter


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))] if v else 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", nargs="*", default=["s1_3x3", "s3_3x3", "s3_1x1_in"])
    ap.add_argument("--cfgs", nargs="*", default=["48:1", "51:1", "50:1", "42:1"],
                    help="tile config:split-K pairs (each is tried on every layer it supports)")
    ap.add_argument("--gemm", nargs="*", default=[], help="dense GEMMs MxNxK (hip().linear) instead of conv layers")
    ap.add_argument("--attention", nargs="*", default=[],
                    help="fixed-S attention BxSxH (D = 64, key mask): stamps entry / staged / softmax / PV / stored")
    a = ap.parse_args()
    n = a.batch
    H = hip()
    for shape in a.attention:
        B, S, NH = (int(v) for v in shape.split("x"))
        qkvs = [torch.randn(B, S, 3 * NH * 64, device="cuda").to(BF) for _ in range(8)]
        mask = torch.zeros(B, S, device="cuda")
        attention_report(f"attn{shape}", lambda j: H.attention(qkvs[j], mask, NH, 0.125, None, S, 0))
    if a.attention:
        return
    for shape in a.gemm:
        M, N, K = (int(v) for v in shape.split("x"))
        xs = [torch.randn(M, K, device="cuda").to(BF) for _ in range(8)]
        ws = [(torch.randn(N, K, device="cuda") * 0.05).to(BF) for _ in range(8)]
        outs = [torch.empty(M, N, device="cuda", dtype=BF) for _ in range(8)]
        b = torch.zeros(N, device="cuda")
        for cs in a.cfgs:
            cfg, sp = (int(x) for x in cs.split(":"))
            report(f"gemm{shape}", cfg, sp,
                   lambda j, cfg=cfg, sp=sp: H.linear(xs[j], ws[j], b, None, ACT["none"], cfg, False, 1.0, outs[j], sp))
    for name in a.layers if not a.gemm else []:
        h, cin, cout, k, s, resid = LAYERS[name]
        pad = k // 2
        ho = (h + 2 * pad - k) // s + 1
        kp = -(-(k * k * cin) // 64) * 64
        xs = [torch.randn(n, h, h, cin, device="cuda").to(BF) for _ in range(8)]
        ws = [(torch.randn(cout, kp, device="cuda") * 0.05).to(BF) for _ in range(8)]
        rs = [torch.randn(n, ho, ho, cout, device="cuda").to(BF) for _ in range(8)] if resid else [None] * 8
        outs = [torch.empty(n, ho, ho, cout, device="cuda", dtype=BF) for _ in range(8)]
        b = torch.zeros(cout, device="cuda")
        for cs in a.cfgs:
            cfg, sp = (int(x) for x in cs.split(":"))
            report(name, cfg, sp, lambda j, cfg=cfg, sp=sp: H.conv2d(
                xs[j], ws[j], b, rs[j], k, k, s, s, pad, pad, pad, pad, ACT["relu"], cfg, outs[j], False, sp))


def attention_report(name, run):
    """Phases of the fixed-S attention kernel (kernels/attention.hip stamps)."""
    H = hip()
    for j in range(8):
        run(j)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for j in range(7):
        run(j)
    e0.record()
    run(7)
    e1.record()
    e1.synchronize()
    ev_us = e0.elapsed_time(e1) * 1e3
    tr = torch.zeros(1 << 20, 8, dtype=torch.int64, device="cuda")
    for j in range(7):
        run(j)
    H.set_wg_trace(tr)
    run(7)
    H.set_wg_trace(None)
    torch.cuda.synchronize()
    t = tr.cpu()
    t = t[t[:, 0] > 0]
    t0 = int(t[:, 0].min())
    ph = {"start": ((t[:, 0] - t0).double() * TICK_US).tolist()}
    for k, nm in ((1, "staged"), (2, "softmax"), (3, "pv"), (4, "stored")):
        ph[nm] = ((t[:, k] - t[:, k - 1]).double() * TICK_US).tolist()
    ph["life"] = ((t[:, 4] - t[:, 0]).double() * TICK_US).tolist()
    per_cu = {}
    for c in t[:, 7].tolist():
        per_cu[c] = per_cu.get(c, 0) + 1
    print(json.dumps({"layer": name, "workgroups": int(t.shape[0]), "event_us": round(ev_us, 2),
                      "span_us": round(float((t[:, 4].max() - t0) * TICK_US), 2), "cus": len(per_cu),
                      "max_wg_per_cu": max(per_cu.values()),
                      **{k: {"p50": round(q(v, .5), 2), "p90": round(q(v, .9), 2), "max": round(max(v), 2)}
                         for k, v in ph.items()}}), flush=True)


def report(name, cfg, sp, run):
    H = hip()
    try:
        for j in range(8):
            run(j)
        torch.cuda.synchronize()
    except RuntimeError as e:
        print(json.dumps({"layer": name, "cfg": cfg, "splits": sp, "error": str(e)[:100]}), flush=True)
        return
    # untraced event time of the same launch (copy 7 after 0..6)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for j in range(7):
        run(j)
    e0.record()
    run(7)
    e1.record()
    e1.synchronize()
    ev_us = e0.elapsed_time(e1) * 1e3
    tr = torch.zeros(1 << 20, 8, dtype=torch.int64, device="cuda")
    for j in range(7):
        run(j)
    H.set_wg_trace(tr)
    run(7)
    H.set_wg_trace(None)
    torch.cuda.synchronize()
    t = tr.cpu()
    t = t[t[:, 0] > 0]
    # split-K slices that are not their tile's last arriver leave after the
    # slab store without the exit stamp: their exit = the end of their K loop
    t[:, 3] = torch.where(t[:, 3] > 0, t[:, 3], t[:, 2])
    nwg = int(t.shape[0])
    t0 = int(t[:, 0].min())
    st = ((t[:, 0] - t0).double() * TICK_US).tolist()
    first = ((t[:, 1] - t[:, 0]).double() * TICK_US).tolist()
    loop = ((t[:, 2] - t[:, 1]).double() * TICK_US).tolist()
    epi = ((t[:, 3] - t[:, 2]).double() * TICK_US).tolist()
    life = ((t[:, 3] - t[:, 0]).double() * TICK_US).tolist()
    span = float((t[:, 3].max() - t0) * TICK_US)
    per_cu = {}
    for c in t[:, 7].tolist():
        per_cu[c] = per_cu.get(c, 0) + 1
    print(json.dumps({
        "layer": name, "cfg": cfg, "splits": sp, "workgroups": nwg, "event_us": round(ev_us, 2),
        "span_us": round(span, 2), "cus": len(per_cu), "max_wg_per_cu": max(per_cu.values()),
        "start_us": {"p50": round(q(st, .5), 2), "p90": round(q(st, .9), 2), "max": round(max(st), 2)},
        "first_data_us": {"p50": round(q(first, .5), 2), "p90": round(q(first, .9), 2)},
        "kloop_us": {"p50": round(q(loop, .5), 2), "p90": round(q(loop, .9), 2)},
        "epilogue_us": {"p50": round(q(epi, .5), 2), "p90": round(q(epi, .9), 2)},
        "wg_life_us": {"p50": round(q(life, .5), 2), "p90": round(q(life, .9), 2)},
    }), flush=True)


if __name__ == "__main__":
    main()
