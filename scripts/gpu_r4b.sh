#!/bin/bash
# Round 4, session 2: numerics of the fixed bottleneck tail + weight-stationary
# GEMM + register-B halo; every candidate's time per layer (3x3 and 1x1); the
# engine with the tail fusion on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
scripts/gpu_session.sh \
 "ktests:420:python -u -m pytest tests/test_kernels_gpu.py -q -k 'halo or tail or weight_stationary' --timeout 120 --timeout-method thread" \
 "sweep3:300:python scripts/conv_sweep.py --layers s2_3x3 s3_3x3 s4_3x3 --top 40" \
 "sweep1:300:python scripts/conv_sweep.py --layers s1_1x1_in s1_1x1_out s2_1x1_in s2_1x1_out s3_1x1_in s3_1x1_out s4_1x1_in s4_1x1_out --top 12" \
 "engine_tail:300:TFSERVE_TAIL=1 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "engine:300:python scripts/bench_engine.py --model resnet50 --batch 1 32"
