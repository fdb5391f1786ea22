"""Per-kernel time of the LAST window of a rocprofv3 kernel trace: the
kernels dispatched after the final tuning marker (the tuner's GPU spin /
L2-flush kernels), i.e. the timed replays of probe_concurrency.py.  Prints
the window's wall span, the summed kernel time, and per kernel: calls,
total / average us and share (durations of concurrent kernels overlap, so
the sum can exceed the span: that excess is the concurrency).

    python scripts/trace_window.py /tmp/kt3 --batches 180
"""
import argparse
import glob
import sqlite3


def short(n: str) -> str:
    n = n.replace("tfsk::", "").replace("(anonymous namespace)::", "").replace("cgemm_impl::", "")
    return n.split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--batches", type=int, default=0, help="batches replayed in the window (per-batch figures)")
    ap.add_argument("--markers", nargs="*", default=["spin_kernel", "FillFunctor"])
    a = ap.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(a.db + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    last = max((i for i, r in enumerate(rows) if any(m in r[0] for m in a.markers)), default=-1)
    win = rows[last + 1:]
    if not win:
        print("empty window")
        return
    span = (max(r[2] for r in win) - min(r[1] for r in win)) / 1e3
    tot = {}
    for n, s, e in win:
        k = short(n)
        t = tot.setdefault(k, [0, 0.0])
        t[0] += 1
        t[1] += (e - s) / 1e3
    busy = sum(v[1] for v in tot.values())
    nb = max(1, a.batches)
    print(f"window: {len(win)} dispatches, span {span:.1f} us, kernel time {busy:.1f} us "
          f"(x{busy / max(span, 1e-9):.2f} overlap)" + (f"; per batch: span {span / nb:.1f} us, kernel "
                                                          f"{busy / nb:.1f} us" if a.batches else ""))
    print("| calls | total us | per batch us | avg us | share | kernel |\n|---|---|---|---|---|---|")
    for k, (cnt, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"| {cnt} | {t:.1f} | {t / nb:.1f} | {t / cnt:.2f} | {100 * t / busy:.1f}% | `{k}` |")


if __name__ == "__main__":
    main()
