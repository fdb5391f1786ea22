#!/bin/bash
# outputs' D2H inside the bucket graph (TFSERVE_GRAPH_D2H) vs separate SDMA copies: fast-path tests, c=1 breakdown, bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aj
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_fastpath_gpu.py tests/test_resnet_gpu.py > gpurun_out/r3aj/tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  TFSERVE_GRAPH_D2H=$v timeout -k 10 300 python -u scripts/c1_breakdown.py > gpurun_out/r3aj/c1_d2h$v.log 2>&1 || exit 1
  echo "d2h=$v $(grep '^{' gpurun_out/r3aj/c1_d2h$v.log)"
done
for v in 1 0; do
  TFSERVE_GRAPH_D2H=$v timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3aj/bench_d2h$v.log 2>&1 || exit 1
  echo "d2h=$v bench $(grep -h '^{' gpurun_out/r3aj/bench_d2h$v.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p50_c1_ms"])')"
done
