#!/bin/bash
# Flow kernel: GPU tests, then engine timing with / without it on the same box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3v
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_flow_gpu.py > gpurun_out/r3v/flow_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 > gpurun_out/r3v/engine_flow.log 2>&1 &&
TFSERVE_FLOW=0 timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 > gpurun_out/r3v/engine_noflow.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r3v/resnet_tests.log 2>&1
