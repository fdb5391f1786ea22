#!/bin/bash
# with 8 (and 12) hardware queues: how many concurrent replays pay (ResNet-50 b32, BERT-base b32)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3am
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u scripts/probe_concurrency.py --lanes 6 > gpurun_out/r3am/probe_q8_l6.log 2>&1 &&
GPU_MAX_HW_QUEUES=12 timeout -k 10 400 python -u scripts/probe_concurrency.py --lanes 6 > gpurun_out/r3am/probe_q12_l6.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u scripts/probe_concurrency.py --model bert-base --lanes 5 > gpurun_out/r3am/probe_bert_q8_l5.log 2>&1 &&
GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python -u scripts/probe_concurrency.py --model bert-base --lanes 5 > gpurun_out/r3am/probe_bert_q4_l5.log 2>&1
for f in gpurun_out/r3am/*.log; do echo "$(basename $f) $(grep -h ms_per_batch $f | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print({k[13:]: v for k, v in d.items() if k.startswith("ms_per_batch")})')"; done
