#!/bin/bash
# 4 vs 8 hardware queues on the other configs (BERT-base, ResNet-50 v2, config 5), interleaved on one box
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ap
for m in bert-base resnet50-v2; do
  for q in 4 8 4 8; do
    TFSERVE_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --model $m --steps 300 --warmup 30 > gpurun_out/r3ap/b_${m}_q$q.log 2>&1 || exit 1
    echo "$m q=$q $(grep -h '^{' gpurun_out/r3ap/b_${m}_q$q.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_latency_ms"], d["p99_latency_ms"])')"
  done
done
for q in 4 8; do
  TFSERVE_HW_QUEUES=$q timeout -k 10 600 python -u bench.py --model multi --steps 300 --warmup 30 > gpurun_out/r3ap/multi_q$q.log 2>&1 || exit 1
  echo "multi q=$q $(grep -h '^{' gpurun_out/r3ap/multi_q$q.log | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["bert_rps"], d["resnet_p99_ms_steady"], d["resnet_p99_ms_during_reload"])')"
done
