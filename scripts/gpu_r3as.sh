#!/bin/bash
# is the headline bound by the load generator's threads? --client-threads 4 (default) vs 6 vs 8, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3as
for rep in 1 2; do
  for t in 4 6 8; do
    timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --client-threads $t > gpurun_out/r3as/bench_t${t}_$rep.log 2>&1 || exit 1
    echo "threads=$t rep=$rep $(grep -h '^{' gpurun_out/r3as/bench_t${t}_$rep.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); c=d.get("cpu_cores_by_thread") or {}; print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["gpu_busy_pct"][0]["mean"], c.get("tfs-loadgen"), c.get("tfs-h2io"), c.get("process_total"))')"
  done
done
