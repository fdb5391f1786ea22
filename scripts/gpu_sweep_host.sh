#!/bin/bash
# Interleaved host-side knobs of the 1-GPU headline bench on one box: distinct request bodies x IO threads.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/sweep_host.log
: > $out
for rep in 1 2; do
  for cfg in "64 6" "8 6" "64 4" "8 4"; do
    set -- $cfg
    echo "== rep=$rep distinct=$1 io=$2" >> $out
    timeout -k 10 150 python -u bench.py --steps 300 --warmup 30 --distinct-requests $1 --io-threads $2 --ref-client-requests 0 --c1-requests 0 --cpu-report >> $out 2>&1 || exit 1
  done
done
