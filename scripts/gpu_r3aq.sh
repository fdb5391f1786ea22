#!/bin/bash
# eager H2D (rows copied to the device as they complete, TFSERVE_EAGER_H2D=1) vs the batched H2D, with 8 HW queues
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aq
i=0
for e in 0 1 0 1 0 1; do
  i=$((i+1))
  TFSERVE_EAGER_H2D=$e timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3aq/bench_e${e}_$i.log 2>&1 || exit 1
  echo "eager=$e run=$i $(grep -h '^{' gpurun_out/r3aq/bench_e${e}_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d.get("cpu_cores_by_thread") or {}; print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["gpu_busy_pct"][0]["mean"], c.get("tfs-nlane"))')"
done
