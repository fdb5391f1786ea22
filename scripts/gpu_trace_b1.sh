#!/bin/bash
# Kernel-trace replay table of the ResNet-50 graph at batch $BATCH (default 1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODEL=${MODEL:-resnet50}
BATCH=${BATCH:-1}
FIRST=${FIRST:-ingest}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_b -o run -- python scripts/bench_engine.py --model $MODEL --batch $BATCH --iters 20 > /tmp/kt_b.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_b -name '*.db' | head -1) --first $FIRST --list > gpurun_out/replay_${MODEL}_b${BATCH}.txt
rc=$?
rm -rf /tmp/prof_b
exit $rc
