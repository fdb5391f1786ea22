#!/bin/bash
# Round 4, session 23: the window's load-generator connections closed before
# the reference-client phase.  2000 steps x2 and the driver command.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4w
mkdir -p $D
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/drv1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000b.log 2>&1
rc=$?
python - <<'PY'
import json
for f in ("b2000a", "drv1", "b2000b"):
    try:
        d = json.loads(open(f"gpurun_out/r4w/{f}.log").read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "n/a", e); continue
    r = d["diagnostics"][0]["ref_client"]
    print(f, d["value"], d["p50_c1_ms"], d["ref_client_rps"], round(d["ref_client_rps"] / d["value"], 2),
          r["tfs-h2io"], r["io_us_per_req_recv"], r["avg_batch"], d["diagnostics"][0]["placement"]["cpus"])
PY
exit $rc
