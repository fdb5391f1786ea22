#!/bin/bash
# Same-box A/B of the fused stem on the GPU-side serving ceiling (concurrent lanes, no network).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for f in 1 0 1 0; do
  echo "== TFSERVE_STEM_POOL=$f" >> gpurun_out/stem_lanes_ab.log
  TFSERVE_STEM_POOL=$f timeout -k 10 300 python -u scripts/bench_lanes.py --batch 32 --lanes 1 4 2>/dev/null | grep "{" >> gpurun_out/stem_lanes_ab.log || exit 1
done
