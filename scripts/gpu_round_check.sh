#!/bin/bash
# Kernel tests + ResNet e2e tests + engine timing + one kernel-trace replay table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODEL=${MODEL:-resnet50}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "classifier or halo or attention" > gpurun_out/chk_kernels.log 2>&1 &&
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/chk_resnet.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model $MODEL --batch 1 32 > gpurun_out/chk_engine.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model $MODEL --batch 32 --iters 20 > /tmp/kt.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt -name '*.db' | head -1) --first ingest --list > gpurun_out/chk_replay_${MODEL}.txt
rc=$?
rm -rf /tmp/prof_kt
exit $rc
