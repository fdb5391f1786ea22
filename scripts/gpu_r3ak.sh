#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES 4 = the box default, vs 8), 4 lanes, interleaved x3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ak
i=0
for q in 4 8 4 8 4 8; do
  i=$((i+1))
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3ak/bench_q${q}_$i.log 2>&1 || exit 1
  echo "q=$q run=$i $(grep -h '^{' gpurun_out/r3ak/bench_q${q}_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"], d["gpu_busy_pct"][0]["mean"])')"
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3ak/probe_q8.log 2>&1 &&
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3ak/probe_q4.log 2>&1
for q in 8 4; do echo "probe q=$q $(grep -h ms_per_batch gpurun_out/r3ak/probe_q$q.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if k.startswith("ms_per_batch")})')"; done
