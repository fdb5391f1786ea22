#!/bin/bash
# Round 4 HEAD check: full GPU suite, smoke, the driver's 1-GPU command, a
# 2000-step bench, the engine (ResNet-50 b1/b32, BERT b32).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4check
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/driver20.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 2000 --warmup 100 > $D/bench2000.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > $D/engine.log 2>&1
rc=$?
tail -3 $D/gpu_suite.log
grep -h '^{' $D/driver20.log $D/bench2000.log $D/engine.log | cut -c1-220
exit $rc
