#!/bin/bash
# one-GPU multi-rank rehearsal: hardware queues scaled by ranks per GPU (new default) vs 8 per process
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3az
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r3az/self2_q4.log 2>&1 &&
TFSERVE_HW_QUEUES=8 TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r3az/self2_q8.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 100 --warmup 10 > gpurun_out/r3az/self4_q2.log 2>&1
rc=$?
for f in self2_q4 self2_q8 self4_q2; do
  grep -h '^{' gpurun_out/r3az/$f.log | python -c '
import sys, json
d = json.loads(sys.stdin.read()); c = d["cpu_cores_by_thread"]
print("'$f'", d["n_gpus"], d["value"], "errors", d["errors"], "end_sync_ms", c.get("end_sync_ms"), "ref_client", d.get("ref_client_rps"))' || true
done
exit $rc
