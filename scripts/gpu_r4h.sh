#!/bin/bash
# Round 4, session 8: workgroup phase traces of the BERT-base b32 GEMMs
# (QKV, FFN1, FFN2, O-proj at M = 4096) over the big-tile cgemm configs.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "traceg:300:python scripts/wg_trace.py --gemm 4096x2304x768 4096x3072x768 4096x768x3072 4096x768x768 --cfgs 72:1 32:1 96:1 39:1 45:1 105:1 37:1 38:1"
