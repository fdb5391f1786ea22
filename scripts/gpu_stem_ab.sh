#!/bin/bash
# Same-box A/B of the fused stem (TFSERVE_STEM_POOL) on the 1-GPU serving bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for f in 1 0 1 0; do
  echo "== TFSERVE_STEM_POOL=$f" >> gpurun_out/stem_ab.log
  TFSERVE_STEM_POOL=$f timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 2>/dev/null | tail -1 >> gpurun_out/stem_ab.log || exit 1
done
