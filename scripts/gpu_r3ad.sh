#!/bin/bash
# are the lane H2D copies SDMA transfers or blit kernels? kernel + memory-copy trace of the concurrency probe
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ad
cd /tmp && rm -rf /tmp/prof_cp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/prof_cp -o run -- python scripts/probe_concurrency.py --iters 20 > gpurun_out/r3ad/probe.log 2>&1 &&
find /tmp/prof_cp -name '*stats*.csv' -exec cp {} gpurun_out/r3ad/ \; &&
ls -la gpurun_out/r3ad
rc=$?
rm -rf /tmp/prof_cp
exit $rc
