"""Per-kernel PMC counter averages from a rocprofv3 --pmc run (rocpd sqlite).

    python scripts/pmc_summary.py /tmp/prof_pmc                 # averages per kernel name
    python scripts/pmc_summary.py /tmp/prof_pmc --replay ingest  # one graph replay, per dispatch

``--replay FIRST`` lists the dispatches of the last complete replay (between the
last two launches of the kernel whose name contains FIRST) in order, one row
per layer, with MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
kernel cycles), kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums GRBM over
the 8 XCDs; MI355X_MICROARCH.md 'DVFS give-back').
"""
import argparse
import glob
import sqlite3
from collections import defaultdict


def _short(k: str) -> str:
    return k.replace("void ", "").replace("tfsk::(anonymous namespace)::", "").split("(tfsk")[0].split("(")[0][:60]


def _columns(c, table):
    return [r[1] for r in c.execute(f"pragma table_info({table})")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--replay", default=None, help="substring of the replay's first kernel")
    a = ap.parse_args()
    dbs = glob.glob(a.path + "/**/*.db", recursive=True) if not a.path.endswith(".db") else [a.path]
    per_dispatch = {}        # (db, dispatch) -> [name, {counter: value}]
    for db in dbs:
        c = sqlite3.connect(db)
        tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
        if "counters_collection" not in tabs:
            print("tables:", tabs)
            return
        cols = _columns(c, "counters_collection")
        did = "dispatch_id" if "dispatch_id" in cols else ("correlation_id" if "correlation_id" in cols else None)
        sel = f"kernel_name, counter_name, value, {did}" if did else "kernel_name, counter_name, value, rowid"
        for k, n, v, d in c.execute(f"select {sel} from counters_collection"):
            ent = per_dispatch.setdefault((db, d), [k, defaultdict(float)])
            ent[1][n] += v
    if a.replay is None:
        agg = defaultdict(lambda: defaultdict(list))
        for k, d in per_dispatch.values():
            for n, v in d.items():
                agg[k][n].append(v)
        for k, d in sorted(agg.items()):
            vals = " ".join(f"{n}={sum(v)/len(v):.4g}" for n, v in sorted(d.items()))
            print(f"{_short(k)}: {vals}")
        return
    rows = [per_dispatch[key] for key in sorted(per_dispatch, key=lambda x: (x[0], x[1]))]
    idx = [i for i, (k, _d) in enumerate(rows) if a.replay in k]
    if len(idx) < 2:
        raise SystemExit(f"need two dispatches of {a.replay!r}, found {len(idx)}")
    rep = rows[idx[-2]:idx[-1]]
    sq = {"GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"}
    have = {n for _k, d in rep for n in d}
    # memory / instruction counters: per dispatch (FETCH_SIZE / WRITE_SIZE are KB in rocprofv3) and totals
    extra = sorted(have - sq)
    util_cols = "SQ_VALU_MFMA_BUSY_CYCLES" in have
    head = f"{'#':>3} {'kernel':60s} {'kcycles':>9}"
    if util_cols:
        head += f" {'mfma%':>6} {'wait%':>6} {'active%':>7}"
    mem = [n for n in ("FETCH_SIZE", "WRITE_SIZE") if n in have]
    # FETCH_SIZE reads 1/2 of the bytes of wide streaming loads on gfx950
    # (MI355X_MICROARCH.md, HBM): doubled here; WRITE_SIZE is exact for 16-B stores
    scale = {"FETCH_SIZE": 2.0, "WRITE_SIZE": 1.0}
    for n in mem:
        head += f" {n[:5] + '_MB':>9} {n[:5] + '_GB/s':>11}"
    print(head + "".join(f" {n:>14}" for n in extra))
    tot = defaultdict(float)
    tot_busy = tot_cyc = 0.0
    for i, (k, d) in enumerate(rep):
        cyc = d.get("GRBM_GUI_ACTIVE", 0.0) / 8
        tot_cyc += cyc
        line = f"{i:3d} {_short(k):60s} {cyc / 1e3:9.1f}"
        if util_cols:
            busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
            tot_busy += busy
            wc = d.get("SQ_WAVE_CYCLES", 0.0)
            util = busy / (1024 * cyc) if cyc else 0.0
            wait = d.get("SQ_WAIT_ANY", 0.0) / wc if wc else 0.0
            act = d.get("SQ_ACTIVE_INST_ANY", 0.0) / wc if wc else 0.0
            line += f" {100 * util:6.1f} {100 * wait:6.1f} {100 * act:7.1f}"
        for n in mem:
            mb = d.get(n, 0.0) * scale[n] / 1024.0          # rocprofv3 reports KB
            # kcycles at the profiled clock (~2.1 GHz under counters: 'DVFS give-back' item 2)
            gbs = mb / 1024.0 / (cyc / 2.1e9) if cyc else 0.0
            line += f" {mb:9.2f} {gbs:11.0f}"
        for n in extra:
            tot[n] += d.get(n, 0.0)
        print(line + "".join(f" {d.get(n, 0.0):14.1f}" for n in extra))
    summary = f"replay: {len(rep)} dispatches, {tot_cyc / 1e3:.1f} kcycles"
    if util_cols:
        summary += f", MFMA busy {100 * tot_busy / (1024 * tot_cyc) if tot_cyc else 0:.1f}% of SIMD-cycles"
    if extra:
        summary += "; totals: " + ", ".join(f"{n}={tot[n]:.1f}" for n in extra)
    print(summary)


if __name__ == "__main__":
    main()
