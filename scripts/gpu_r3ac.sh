#!/bin/bash
# chained stage-2 1x1 pairs under the serving regime (concurrent lanes) vs default, interleaved
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ac
for v in default all default all; do
  if [ $v = all ]; then export TFSERVE_CONV_CHAIN_SHAPES=all; else unset TFSERVE_CONV_CHAIN_SHAPES; fi
  timeout -k 10 300 python -u scripts/probe_concurrency.py > gpurun_out/r3ac/probe_$v.log 2>&1 || exit 1
  echo "$v $(grep -h ms_per_batch gpurun_out/r3ac/probe_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if k.startswith("ms_per_batch")})')"
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3ac/bench_$v.log 2>&1 || exit 1
  echo "$v bench $(grep -h '^{' gpurun_out/r3ac/bench_$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"])')"
done
