#!/bin/bash
# Stem kernel ablations (TFSK_STEM_DBG bits: 1 loads, 2 MFMAs, 4 pool, 8 conv-tile stores), eager timing.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/stem_ablate.log
: > $out
for d in 0 1 2 4 8 3 7 15 0; do
  echo "== TFSK_STEM_DBG=$d" >> $out
  TFSK_STEM_DBG=$d timeout -k 10 60 python -u scripts/stem_bench.py --batch 32 --iters 100 >> $out 2>&1 || exit 1
  TFSK_STEM_DBG=$d timeout -k 10 60 python -u scripts/stem_bench.py --batch 1 --iters 100 >> $out 2>&1 || exit 1
done
