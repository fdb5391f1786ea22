#!/bin/bash
# Round 4, session 25: small buckets write the head's rows straight into the
# lane's pinned outputs (no D2H blits).  Head / ResNet / fast-path GPU tests,
# the b1 runner path's kernel list, c1, the driver command and 2000 steps.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4y
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_resnet_gpu.py tests/test_kernels_gpu.py tests/test_fastpath_gpu.py -m gpu -x -q -k 'host or classifier or resnet or fastpath or native or lane' --timeout 200 --timeout-method thread > $D/tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1.log 2>&1 &&
TFSERVE_HEAD_HOST=0 timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1_off.log 2>&1 &&
timeout -k 10 200 python -u scripts/c1_breakdown.py > $D/c1_b.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 > /tmp/kt1.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt1 -name '*.db' | head -1) --first stem_pool --list > $D/replay_r50_b1_runpath.txt &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/drv1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/b2000.log 2>&1
rc=$?
rm -rf /tmp/prof_kt1
tail -2 $D/tests.log
for f in c1 c1_off c1_b; do echo "$f $(tail -1 $D/$f.log | cut -c1-120)"; done
tail -4 $D/replay_r50_b1_runpath.txt
grep -h '^{' $D/drv1.log $D/b2000.log | cut -c1-160
exit $rc
