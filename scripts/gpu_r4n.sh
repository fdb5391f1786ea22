#!/bin/bash
# Round 4, session 14: the driver's command twice (reference-client window
# now 20000 calls).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "drv1:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "drv2:300:python bench.py --gpus 1 --steps 20 --warmup 5"
