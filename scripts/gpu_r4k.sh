#!/bin/bash
# Round 4, session 11: split-K fixup with the last arriver's slab loads batched
# (4 slices per round, chunks unrolled): numerics, b1 / b32 split traces,
# engine with the fixup off / on (alternating).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "ktests:400:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'splitk or halo or cgemm' --timeout 120 --timeout-method thread" \
 "b1split:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --batch 1 --layers s3_3x3 s4_3x3 s4_1x1_in --cfgs 51:1 51:4 54:4 36:1 36:4" \
 "trace4:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --layers s4_3x3 s3_3x3 --cfgs 54:1 48:4 50:4 51:2" \
 "eng_on:300:TFSERVE_SPLITK_FIXUP=1 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_off:300:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_on2:300:TFSERVE_SPLITK_FIXUP=1 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_off2:300:python scripts/bench_engine.py --model resnet50 --batch 1 32"
