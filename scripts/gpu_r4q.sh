#!/bin/bash
# Round 4, session 17: one-launch head with its weight / bias loads issued
# ahead of the pooling.  Head tests, engine b1/b32 A/B, b1 replay list, c1.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4q
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -k 'classifier' --timeout 120 --timeout-method thread > $D/tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > $D/engine_fused.log 2>&1 &&
TFSERVE_HEAD_FUSED=0 timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > $D/engine_3launch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 > /tmp/kt1.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt1 -name '*.db' | head -1) --first stem_pool --list > $D/replay_r50_b1.txt &&
timeout -k 10 300 python -u scripts/c1_breakdown.py > $D/c1.log 2>&1 &&
TFSERVE_HEAD_FUSED=0 timeout -k 10 300 python -u scripts/c1_breakdown.py > $D/c1_3launch.log 2>&1
rc=$?
rm -rf /tmp/prof_kt1
tail -3 $D/tests.log
grep -h '^{' $D/engine_fused.log $D/engine_3launch.log | cut -c1-200
head -1 $D/replay_r50_b1.txt; grep head_small $D/replay_r50_b1.txt | head -1 | cut -c1-80; tail -1 $D/c1.log; tail -1 $D/c1_3launch.log
exit $rc
