#!/bin/bash
# Round 4, session 26: 2-rank gloo rehearsal of --gpus 2 on one GPU after the
# transport changes (one acceptor per process, window connections closed
# before the reference-client phase, host-row head).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4z
mkdir -p $D
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 1000 --warmup 50 > $D/gloo2.log 2>&1
rc=$?
python - <<'PY'
import json
try:
    d = json.loads([l for l in open("gpurun_out/r4z/gloo2.log") if l.startswith("{")][-1])
    print(d["value"], d["n_gpus"], d.get("rccl_ok"), d.get("rccl_problems"), d["ref_client_rps"], d.get("ref_client_gpu_share"), d["p50_c1_ms"])
except Exception as e:
    print("n/a", e)
PY
tail -3 $D/gloo2.log | cut -c1-300
exit $rc
