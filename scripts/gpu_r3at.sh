#!/bin/bash
# headline distribution on one box: the driver's exact command (20 steps) and 300-step runs, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3at
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3at/driver_$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3at/long_$i.log 2>&1 || exit 1
  echo "run=$i driver20 $(grep -h '^{' gpurun_out/r3at/driver_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])') long300 $(grep -h '^{' gpurun_out/r3at/long_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
