#!/bin/bash
# Round 4, first GPU session: new kernels' numerics (register-B halo, bottleneck
# tail, split-K counter release), engine timing with / without the tail fusion,
# the 3x3 layer sweep, the transport-only probe and the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scripts/gpu_session.sh \
 "ktests:420:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'halo or splitk or tail' --timeout 120 --timeout-method thread" \
 "engine:240:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "engine_tail:300:TFSERVE_TAIL=1 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "sweep:300:python scripts/conv_sweep.py --layers s2_3x3 s3_3x3 s4_3x3 --top 6" \
 "tiny1:200:python bench.py --model tiny --steps 2000 --warmup 100" \
 "r50:200:python bench.py --steps 2000 --warmup 100"
