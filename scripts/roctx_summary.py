"""Summarise roctx ranges + kernels from a rocprofv3 run (rocpd sqlite):
per-range-name count / mean / p50 / p99 host duration (the native lanes'
tfs.batch / tfs.issue / tfs.gpu_wait, the Python path's tfs.rpc / tfs.batch)
next to the per-kernel totals.  Run on the GPU box right after the profile so
only this text travels back."""
import glob
import json
import sqlite3
import sys


def pct(v, q):
    return v[min(len(v) - 1, int(q * len(v)))] if v else 0.0


def main():
    path = sys.argv[1] if sys.argv[1].endswith(".db") else glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    objs = [r[0] for r in c.execute("select name from sqlite_master where type in ('view','table')")]
    print(f"source: {path}")
    region = next((t for t in ("regions", "regions_and_samples") if t in objs), None)
    if region:
        cols = [r[1] for r in c.execute(f"pragma table_info({region})")]
        cat = "category" if "category" in cols else None
        q = f"select name, duration, {cat or 'NULL'}, {'extdata' if 'extdata' in cols else 'NULL'} from {region}"
        by = {}
        shown = False
        for row in c.execute(q):
            if cat and "MARKER" not in str(row[2]).upper():
                continue
            msg = row[0]
            if row[3]:                       # roctx message: in extdata JSON for rocpd
                try:
                    ext = json.loads(row[3])
                    msg = ext.get("message") or ext.get("msg") or next(
                        (v for v in ext.values() if isinstance(v, str) and v.startswith("tfs.")), msg)
                except (ValueError, AttributeError):
                    pass
                if not shown:
                    print(f"(extdata example: {str(row[3])[:160]})")
                    shown = True
            key = msg.split(" ep=")[0].split(" rows=")[0]
            by.setdefault(key, []).append(row[1] / 1e3)
        print("\n| roctx range | count | mean us | p50 us | p99 us |\n|---|---|---|---|---|")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            v.sort()
            print(f"| {k} | {len(v)} | {sum(v)/len(v):.1f} | {pct(v, .5):.1f} | {pct(v, .99):.1f} |")
    else:
        print("no region view; objects:", objs)
    rows = c.execute("select name, count(*), sum(duration) from kernels group by name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    print("\n| kernel | calls | total us | share |\n|---|---|---|---|")
    for n, k, s in rows[:20]:
        print(f"| {n[:90]} | {k} | {s/1e3:.1f} | {100*s/tot:.1f}% |")


if __name__ == "__main__":
    main()
