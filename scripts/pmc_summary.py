"""Per-kernel PMC counter averages from a rocprofv3 --pmc run (rocpd sqlite or counter CSV)."""
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    agg = defaultdict(lambda: defaultdict(list))
    for db in dbs:
        c = sqlite3.connect(db)
        tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
        if "counters_collection" in tabs:
            q = "select kernel_name, counter_name, value from counters_collection"
        else:
            print("tables:", tabs)
            return
        for k, n, v in c.execute(q):
            agg[k][n].append(v)
    for k, d in sorted(agg.items()):
        short = k.replace("void ", "").replace("tfsk::(anonymous namespace)::", "").split("(tfsk")[0][:70]
        vals = " ".join(f"{n}={sum(v)/len(v):.4g}" for n, v in sorted(d.items()))
        print(f"{short}: {vals}")


if __name__ == "__main__":
    main()
