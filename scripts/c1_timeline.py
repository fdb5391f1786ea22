"""Device-side timeline of concurrency-1 batches from a rocprofv3
`--kernel-trace --memory-copy-trace` database (rocpd sqlite): per batch, the
H2D copy, the gap from the copy's end to the graph's first kernel, the
graph's span, and the D2H copies after it.  Medians over the batches.

    rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/c1 -o run -- python scripts/c1_breakdown.py
    python scripts/c1_timeline.py /tmp/c1
"""
import argparse
import glob
import json
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--min-kernels", type=int, default=20, help="kernels a batch's graph has at least")
    a = ap.parse_args()
    path = a.path if a.path.endswith(".db") else sorted(glob.glob(a.path + "/**/*.db", recursive=True))[-1]
    c = sqlite3.connect(path)
    names = {r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")}
    kern = c.execute("select start, end from kernels order by start").fetchall()
    copies = []
    for view in ("memory_copies", "memory_copy"):
        if view in names:
            cols = [r[1] for r in c.execute(f"pragma table_info({view})")]
            kind = "direction" if "direction" in cols else ("name" if "name" in cols else None)
            q = f"select start, end, {kind or repr('?')}, {'size' if 'size' in cols else 0} from {view} order by start"
            copies = c.execute(q).fetchall()
            break
    h2d = [(s, e, sz) for s, e, k, sz in copies if "HOST_TO_DEVICE" in str(k).upper() or "H2D" in str(k).upper()]
    d2h = [(s, e, sz) for s, e, k, sz in copies if "DEVICE_TO_HOST" in str(k).upper() or "D2H" in str(k).upper()]
    rows = []
    for i, (s, e, sz) in enumerate(h2d):
        nxt = h2d[i + 1][0] if i + 1 < len(h2d) else float("inf")
        ks = [k for k in kern if e <= k[0] < nxt]
        if len(ks) < a.min_kernels:
            continue
        ds = [d for d in d2h if ks[-1][1] <= d[0] < nxt]
        rows.append({"h2d_us": (e - s) / 1e3, "h2d_bytes": sz, "copy_to_kernel_us": (ks[0][0] - e) / 1e3,
                     "graph_span_us": (ks[-1][1] - ks[0][0]) / 1e3,
                     "d2h_us": sum((d[1] - d[0]) for d in ds) / 1e3,
                     "total_us": ((ds[-1][1] if ds else ks[-1][1]) - s) / 1e3})
    out = {"db": path, "views": sorted(n for n in names if not n.startswith("rocpd_"))[:30], "batches": len(rows),
           "h2d_copies": len(h2d), "d2h_copies": len(d2h)}
    for key in ("h2d_us", "copy_to_kernel_us", "graph_span_us", "d2h_us", "total_us"):
        if rows:
            out[key + "_p50"] = round(statistics.median(r[key] for r in rows), 2)
    if rows:
        out["h2d_bytes"] = rows[0]["h2d_bytes"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
