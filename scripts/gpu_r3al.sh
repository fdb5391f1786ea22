#!/bin/bash
# GPU_MAX_HW_QUEUES 4 vs 8 (and 8 with 5 lanes), interleaved x4, 1-GPU headline bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3al
i=0
for rep in 1 2 3 4; do
  for cfg in q4_l4 q8_l4 q8_l5; do
    i=$((i+1))
    q=${cfg:1:1}; l=${cfg:4:1}
    c=$((l*32))
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --lanes $l --concurrency $c > gpurun_out/r3al/bench_${cfg}_$rep.log 2>&1 || exit 1
    echo "$cfg rep=$rep $(grep -h '^{' gpurun_out/r3al/bench_${cfg}_$rep.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["gpu_busy_pct"][0]["mean"])')"
  done
done
