#!/bin/bash
# Same-box A/B of the in-kernel split-K fixup (TFSERVE_SPLITK_FIXUP) on the
# ResNet-50 engine, after checking the kernels with the fixup on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TFSERVE_SPLITK_FIXUP=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fixup_kernels.log 2>&1 || exit 1
for f in 0 1 0 1; do
  echo "== TFSERVE_SPLITK_FIXUP=$f" >> gpurun_out/fixup_ab.log
  TFSERVE_SPLITK_FIXUP=$f timeout -k 10 300 python -u scripts/bench_engine.py --model resnet50 --batch 1 32 >> gpurun_out/fixup_ab.log 2>&1 || exit 1
done
