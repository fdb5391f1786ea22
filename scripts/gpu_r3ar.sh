#!/bin/bash
# kernel statistics of the serving regime itself: rocprofv3 kernel + memory-copy trace over a short 1-GPU bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3ar
rm -rf /tmp/prof_srv
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/prof_srv -o run -- python bench.py --steps 100 --warmup 10 --c1-requests 0 --ref-client-requests 0 > gpurun_out/r3ar/bench.log 2>&1 &&
find /tmp/prof_srv -name '*stats*.csv' -exec cp {} gpurun_out/r3ar/ \;
rc=$?
rm -rf /tmp/prof_srv
exit $rc
