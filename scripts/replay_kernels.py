"""Per-kernel breakdown of ONE steady-state graph replay from a rocprofv3
kernel-trace database: the dispatches between the last two launches of the
replay's first kernel (``--first``), grouped by kernel name.

    python scripts/replay_kernels.py gpurun_out/prof/run_results.db --first embed_ln
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--first", required=True, help="substring of the replay's first kernel name")
    ap.add_argument("--list", action="store_true", help="print every dispatch in order")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x / workgroup_x, grid_y / workgroup_y, grid_z / workgroup_z "
                     "from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.first in r[0]]
    if len(idx) < 2:
        raise SystemExit(f"need two launches of {a.first!r}, found {len(idx)}")
    rep = rows[idx[-2]:idx[-1]]
    span = (rep[-1][2] - rep[0][1]) / 1e3
    busy = sum(r[2] - r[1] for r in rep) / 1e3
    print(f"one replay: {len(rep)} dispatches, span {span:.1f} us, kernel busy {busy:.1f} us")
    if a.list:
        for r in rep:
            print(f"  {(r[2] - r[1]) / 1e3:8.2f} us  wg {r[3]}x{r[4]}x{r[5]}  {r[0][:100]}")
    agg = defaultdict(lambda: [0, 0.0])
    for r in rep:
        agg[r[0]][0] += 1
        agg[r[0]][1] += (r[2] - r[1]) / 1e3
    for name, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:4d} {t:9.1f} us {100 * t / busy:5.1f}%  {name[:100]}")


if __name__ == "__main__":
    main()
