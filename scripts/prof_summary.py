"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) into markdown:
per-kernel totals and, optionally, the per-dispatch sequence of one iteration."""
import argparse
import glob
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--iter-marker", default="", help="kernel-name substring that starts each iteration")
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(a.db + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration) from kernels "
                     "group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows)
    print(f"# {a.title}\n\nsource: `{path}`\n\n| total us | calls | avg us | min us | share | kernel |\n|---|---|---|---|---|---|")
    for n, cnt, s, avg, mn in rows[:30]:
        print(f"| {s/1e3:.1f} | {cnt} | {avg/1e3:.2f} | {mn/1e3:.2f} | {100*s/total:.1f}% | `{short(n)}` |")
    if a.iter_marker:
        seq = c.execute("select name, duration, grid_x, workgroup_x, vgpr_count, lds_size from kernels "
                        "order by start").fetchall()
        idx = [i for i, r in enumerate(seq) if a.iter_marker in r[0]]
        if len(idx) >= 2:
            s, e = idx[-2], idx[-1]
            it = seq[s:e]
            print(f"\n## one iteration ({len(it)} dispatches, {sum(r[1] for r in it)/1e3:.1f} us of kernel time)\n")
            print("| # | us | workgroups | vgpr | lds | kernel |\n|---|---|---|---|---|---|")
            for i, r in enumerate(it):
                print(f"| {i} | {r[1]/1e3:.1f} | {r[2]//max(1,r[3])} | {r[4]} | {r[5]} | `{short(r[0])}` |")


def short(n):
    return n.replace("void ", "").replace("tfsk::(anonymous namespace)::", "").split("(tfsk")[0][:90]


if __name__ == "__main__":
    main()
