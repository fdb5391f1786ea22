#!/bin/bash
# Round 4, session 5: per-workgroup phase traces of the 3x3 (halo) and 1x1
# (cgemm) layers at b32; halo / cgemm numerics after the trace field; one
# SQ PMC pass with the MFMA-busy counter set.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "ktests:300:python -u -m pytest tests/test_kernels_gpu.py -x -q -k 'halo or cgemm_linear' --timeout 120 --timeout-method thread" \
 "trace3:240:python scripts/wg_trace.py --layers s1_3x3 s2_3x3 s3_3x3 s4_3x3 --cfgs 48:1 51:1 50:1 49:1 54:1 56:1" \
 "trace1:240:python scripts/wg_trace.py --layers s1_1x1_out s3_1x1_in s3_1x1_out s4_1x1_in --cfgs 42:1 36:1 43:1 71:1" \
 "pmc:300:timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 --graph-tune 0 && python scripts/pmc_summary.py /tmp/prof_pmc --replay stem_pool > gpurun_out/pmc_r50_b32_mfma.txt"
