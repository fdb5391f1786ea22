#!/bin/bash
# Round 4, session 13: engine A/B of the split-K fixup default (auto: < 128
# tiles) against off, alternating on one box.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "auto1:300:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "off1:300:TFSERVE_SPLITK_FIXUP=0 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "auto2:300:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "off2:300:TFSERVE_SPLITK_FIXUP=0 python scripts/bench_engine.py --model resnet50 --batch 1 32"
