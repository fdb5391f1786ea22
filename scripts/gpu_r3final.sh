#!/bin/bash
# HEAD check: full GPU suite, smoke, 1-GPU bench, engine (R50 b1/b32, BERT b32), b32 replay table
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3final2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3final2/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3final2/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3final2/bench1.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3final2/engine.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model bert-base --batch 32 > gpurun_out/r3final2/engine_bert.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 > /tmp/kt.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt -name '*.db' | head -1) --first stem_pool --list > gpurun_out/r3final2/r50_b32_replay.txt
rc=$?
rm -rf /tmp/prof_kt
[ $rc -eq 0 ] || exit $rc
