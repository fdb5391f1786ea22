"""Kernel mix of the SERVING regime from a rocprofv3 kernel-trace database of a
bench.py run: the dispatches of the busiest ``--window-ms`` stretch (several
batches replaying on the lanes at once), grouped by kernel name.

    rocprofv3 --kernel-trace -d /tmp/kt -o run -- python bench.py --steps 2000 --warmup 100
    python scripts/serving_kernel_mix.py /tmp/kt/.../run_results.db --window-ms 50

Summed kernel durations exceed the wall window when lanes overlap: the ratio
(``overlap``) is the mean number of kernels in flight; each kernel's share of
the summed time approximates its share of the GPU's work in the serving
regime, where the isolated replay tables (scripts/replay_kernels.py) time one
batch alone.
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window-ms", type=float, default=50.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    if not rows:
        raise SystemExit("no kernels in the trace")
    w = int(a.window_ms * 1e6)
    # the window with the most kernel time: slide over dispatch start times
    best, best_i, j, acc = -1, 0, 0, 0
    for i in range(len(rows)):
        while j < len(rows) and rows[j][1] < rows[i][1] + w:
            acc += rows[j][2] - rows[j][1]
            j += 1
        if acc > best:
            best, best_i = acc, i
        acc -= rows[i][2] - rows[i][1]
    t0 = rows[best_i][1]
    sel = [r for r in rows[best_i:] if r[1] < t0 + w]
    wall = (max(r[2] for r in sel) - t0) / 1e3
    total = sum(r[2] - r[1] for r in sel) / 1e3
    print(f"window: {len(sel)} dispatches over {wall:.1f} us wall, summed kernel time {total:.1f} us, "
          f"overlap {total / wall:.2f}")
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in sel:
        agg[name][0] += 1
        agg[name][1] += (e - s) / 1e3
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{n:5d} {t:10.1f} us {100 * t / total:5.1f}%  {t / n:7.2f} us/launch  {name[:96]}")


if __name__ == "__main__":
    main()
