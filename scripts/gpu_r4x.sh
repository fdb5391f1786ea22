#!/bin/bash
# Round 4, session 24: copies on SDMA (default) vs blit kernels
# (HSA_ENABLE_SDMA=0) for the concurrency-1 path and the headline.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4x
mkdir -p $D
timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1_sdma.log 2>&1 &&
HSA_ENABLE_SDMA=0 timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1_blit.log 2>&1 &&
timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1_sdma2.log 2>&1 &&
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000_blit.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000_sdma.log 2>&1
rc=$?
for f in c1_sdma c1_blit c1_sdma2; do echo "$f $(tail -1 $D/$f.log)"; done
python - <<'PY'
import json
for f in ("b2000_blit", "b2000_sdma"):
    try:
        d = json.loads(open(f"gpurun_out/r4x/{f}.log").read().strip().splitlines()[-1])
        print(f, d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["ref_client_rps"])
    except Exception as e:
        print(f, "n/a", e)
PY
exit $rc
