#!/bin/bash
# Round 4, session 20: BERT's K=3072 / N=768 GEMMs (FFN2, attention output)
# with larger tiles split over K, in-kernel fixup on vs separate reduce.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4t
mkdir -p $D
TFSERVE_SPLITK_FIXUP=1 timeout -k 10 300 python -u scripts/wg_trace.py --gemm 4096x768x3072 4096x768x768 --cfgs 105:1 72:4 72:2 37:2 37:3 38:3 39:2 32:2 105:2 45:2 > $D/fix1.log 2>&1 &&
TFSERVE_SPLITK_FIXUP=0 timeout -k 10 300 python -u scripts/wg_trace.py --gemm 4096x768x3072 --cfgs 72:4 37:3 38:3 39:2 105:2 > $D/fix0.log 2>&1
rc=$?
python - <<'PY'
import json
for f in ("gpurun_out/r4t/fix1.log", "gpurun_out/r4t/fix0.log"):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            print(f[-8:], d["layer"], d["cfg"], d["splits"], d.get("workgroups"), d.get("event_us"), d.get("error", ""))
PY
exit $rc
