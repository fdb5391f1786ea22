#!/bin/bash
# batch-1 replay table (per-kernel), default and with the in-kernel split-K fixup
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3af
for v in 0 1; do
  rm -rf /tmp/prof_b1
  TFSERVE_SPLITK_FIXUP=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_b1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 > /tmp/b1.log 2>&1 || exit 1
  python scripts/replay_kernels.py $(find /tmp/prof_b1 -name '*.db' | head -1) --first stem_pool --list > gpurun_out/r3af/r50_b1_replay_fixup$v.txt || exit 1
  TFSERVE_SPLITK_FIXUP=$v timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 2 4 > gpurun_out/r3af/engine_fixup$v.log 2>&1 || exit 1
done
rm -rf /tmp/prof_b1
