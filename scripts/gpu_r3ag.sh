#!/bin/bash
# deep-ring cgemm configs: kernel tests for the new configs, fresh-tuned engine (the committed table's schema
# no longer matches, so every key re-tunes) vs the same tree without the deep-ring candidates
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ag
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "cgemm" > gpurun_out/r3ag/cgemm_tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 32 > gpurun_out/r3ag/engine_deep.log 2>&1 &&
TFSERVE_NO_DEEP_RING=1 timeout -k 10 400 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 32 > gpurun_out/r3ag/engine_nodeep.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 32 > gpurun_out/r3ag/engine_deep2.log 2>&1
