#!/bin/bash
# Round 4, session 21: where BERT's attention kernel spends its 12.6 us
# (per-workgroup phase stamps), at b16 / b32 / b64; attention tests.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/r4u
mkdir -p $D
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k attention --timeout 120 --timeout-method thread > $D/tests.log 2>&1 &&
timeout -k 10 200 python -u scripts/wg_trace.py --attention 32x128x12 16x128x12 64x128x12 8x128x12 > $D/attn.log 2>&1
rc=$?
tail -2 $D/tests.log; cat $D/attn.log
exit $rc
