#!/bin/bash
# Round 4, session 6: the fragment-prefetch (PF) halo configs 80-88 and cgemm
# configs 96-106 -- numerics vs fp32, per-layer sweeps (3x3 and 1x1 at b32,
# 3x3 at b1), workgroup phase traces, engine timing with PF candidates.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "ktests:400:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'halo or cgemm' --timeout 120 --timeout-method thread" \
 "sweep3:300:python scripts/conv_sweep.py --layers s1_3x3 s2_3x3 s3_3x3 s4_3x3 --top 12" \
 "sweep1:300:python scripts/conv_sweep.py --layers s1_1x1_in s1_1x1_out s2_1x1_in s2_1x1_out s3_1x1_in s3_1x1_out s4_1x1_in s4_1x1_out --top 8" \
 "trace3:240:python scripts/wg_trace.py --layers s1_3x3 s2_3x3 s3_3x3 s4_3x3 --cfgs 48:1 80:1 50:1 82:1 51:1 83:1 54:1 86:1" \
 "engine:300:python scripts/bench_engine.py --model resnet50 --batch 1 32"
