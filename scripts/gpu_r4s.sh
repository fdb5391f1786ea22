#!/bin/bash
# Round 4, session 19: current ResNet-50 b32 and BERT-base b32 replay tables
# (kernel trace, one replay's dispatch list).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4s
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_r50 -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 > $D/r50.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_r50 -name '*.db' | head -1) --first stem_pool --list > $D/replay_r50_b32.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_bert -o run -- python scripts/bench_engine.py --model bert-base --batch 32 --iters 20 > $D/bert.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_bert -name '*.db' | head -1) --first embed_ln --list > $D/replay_bert_b32.txt
rc=$?
rm -rf /tmp/prof_r50 /tmp/prof_bert
head -1 $D/replay_r50_b32.txt; head -1 $D/replay_bert_b32.txt
exit $rc
