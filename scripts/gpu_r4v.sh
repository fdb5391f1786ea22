#!/bin/bash
# Round 4, session 22: one acceptor per process hands connections to the IO
# thread with the fewest (was: per-thread SO_REUSEPORT hash).  Fast-path GPU
# tests, the driver command x2 and 2000 steps (reference-client window).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4v
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k 'fastpath or native or lane' --timeout 120 --timeout-method thread > $D/fptests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/drv1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/drv2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000.log 2>&1
rc=$?
tail -1 $D/fptests.log
python - <<'PY'
import json
for f in ("drv1", "drv2", "b2000"):
    try:
        d = json.loads(open(f"gpurun_out/r4v/{f}.log").read().strip().splitlines()[-1])
    except Exception as e:
        print(f, "n/a", e); continue
    r = d["diagnostics"][0]["ref_client"]
    print(f, d["value"], d["p50_c1_ms"], d["ref_client_rps"], round(d["ref_client_rps"] / d["value"], 2),
          r["tfs-h2io"], r["avg_batch"], r["client_threads_cores"])
PY
exit $rc
