#!/bin/bash
# Tiny-kernel graph chain cost under HIP runtime settings (one process each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/launch_floor.log
: > $out
timeout -k 10 60 python -u scripts/launch_floor.py >> $out 2>&1 &&
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 60 python -u scripts/launch_floor.py >> $out 2>&1 &&
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 python -u scripts/launch_floor.py >> $out 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 60 python -u scripts/launch_floor.py >> $out 2>&1 &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 60 python -u scripts/launch_floor.py >> $out 2>&1 &&
timeout -k 10 120 python -u scripts/bench_engine.py --model resnet50 --batch 1 >> $out 2>&1 &&
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python -u scripts/bench_engine.py --model resnet50 --batch 1 >> $out 2>&1
