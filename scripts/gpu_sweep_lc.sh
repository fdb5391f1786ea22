#!/bin/bash
# Interleaved lanes x concurrency sweep of the 1-GPU headline bench on one box (continuous load generator).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/sweep_lc.log
: > $out
for rep in 1 2; do
  for lc in "4 128" "4 192" "6 192" "6 256" "8 256"; do
    set -- $lc
    echo "== rep=$rep lanes=$1 conc=$2" >> $out
    timeout -k 10 150 python -u bench.py --steps 300 --warmup 30 --lanes $1 --concurrency $2 --ref-client-requests 0 --c1-requests 0 --cpu-report >> $out 2>&1 || exit 1
  done
done
