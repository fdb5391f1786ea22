#!/bin/bash
# refresh the per-config serving numbers with 8 hardware queues: BERT-base, ResNet-50 v2, config 5 (multi), headline
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ao
timeout -k 10 300 python -u bench.py --model bert-base --steps 300 --warmup 30 > gpurun_out/r3ao/bench_bert.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model resnet50-v2 --steps 300 --warmup 30 > gpurun_out/r3ao/bench_v2.log 2>&1 &&
timeout -k 10 600 python -u bench.py --model multi --steps 300 --warmup 30 > gpurun_out/r3ao/bench_multi.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3ao/bench_r50.log 2>&1
for f in bert v2 r50; do echo "$f $(grep -h '^{' gpurun_out/r3ao/bench_$f.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p99_latency_ms"], d.get("p50_c1_ms"), d["errors"])')"; done
grep -h '^{' gpurun_out/r3ao/bench_multi.log | tail -1 | cut -c1-600
