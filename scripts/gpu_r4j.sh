#!/bin/bash
# Round 4, session 10: vectorized agent-coherent split-K fixup (16-B sc1
# stores / loads), host-overhead-free tuner timing, whole-image halo tiles
# (TI images per tile on 7x7 maps): numerics, b32 3x3 sweeps with the fixup,
# b1 split traces, engine with the fixup off / on (alternating).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "ktests:400:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'splitk or halo or cgemm' --timeout 120 --timeout-method thread" \
 "sweep3fx:300:TFSERVE_SPLITK_FIXUP=1 python scripts/conv_sweep.py --layers s3_3x3 s4_3x3 --top 10" \
 "b1split:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --batch 1 --layers s2_3x3 s3_3x3 s4_3x3 --cfgs 51:1 51:2 51:4 54:1 54:4" \
 "b1split1:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --batch 1 --layers s3_1x1_in s4_1x1_in s4_1x1_out --cfgs 36:1 36:2 36:4 42:1 42:4" \
 "trace4:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --layers s4_3x3 s3_3x3 --cfgs 54:1 48:1 48:2 48:4 50:2 50:4" \
 "eng_off:300:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_on:300:TFSERVE_SPLITK_FIXUP=1 python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_off2:300:python scripts/bench_engine.py --model resnet50 --batch 1 32" \
 "eng_on2:300:TFSERVE_SPLITK_FIXUP=1 python scripts/bench_engine.py --model resnet50 --batch 1 32"
