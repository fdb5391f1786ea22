#!/bin/bash
# Round 4, session 12: split-K fixup on automatically for launches of < 128
# tiles.  Full GPU suite, smoke, engine b1/b32 (x2), concurrency-1 latency
# via the headline bench.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/${CHECK_DIR:-r4l}
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/driver20.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > $D/engine.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > $D/engine2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/bench2000.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 > /tmp/kt1.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt1 -name '*.db' | head -1) --first stem_pool --list > $D/replay_r50_b1.txt
rc=$?
rm -rf /tmp/prof_kt1
tail -3 $D/gpu_suite.log
grep -h '^{' $D/driver20.log $D/engine.log $D/engine2.log $D/bench2000.log | cut -c1-220
exit $rc
