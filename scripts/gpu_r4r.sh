#!/bin/bash
# Round 4, session 18: weight-replication GPU tests, including the reload
# broadcast against live replaying lanes.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4r
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests/test_weights_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $D/weights.log 2>&1
rc=$?
tail -8 $D/weights.log
exit $rc
