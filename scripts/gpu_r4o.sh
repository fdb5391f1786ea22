#!/bin/bash
# Round 4, session 15: completion tail spun for small buckets -- the fast-path
# GPU tests, concurrency-1 latency (c1 breakdown) and the headline twice.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "fptests:400:python -u -m pytest tests -m gpu -x -q -k 'fastpath or native or lane' --timeout 120 --timeout-method thread" \
 "c1:300:python scripts/c1_breakdown.py" \
 "drv1:300:python bench.py --gpus 1 --steps 20 --warmup 5" \
 "b2000:300:python bench.py --steps 2000 --warmup 100"
