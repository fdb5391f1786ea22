#!/bin/bash
# Round 4, session 9: the serving regime.  Concurrency probe (ResNet-50 b32,
# 1..4 batches in flight) with the default graph tuner and with a wider
# candidate set (top 12 within 2.5x of the isolated best); the headline with
# each, interleaved on one box.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "conc_def:300:python scripts/probe_concurrency.py --model resnet50 --batch 32 --lanes 4" \
 "conc_wide:400:TFSERVE_GRAPH_TUNE_TOP=12 TFSERVE_GRAPH_TUNE_RATIO=2.5 python scripts/probe_concurrency.py --model resnet50 --batch 32 --lanes 4" \
 "b_def1:200:python bench.py --steps 2000 --warmup 100 --ref-client-requests 0" \
 "b_wide1:300:TFSERVE_GRAPH_TUNE_TOP=12 TFSERVE_GRAPH_TUNE_RATIO=2.5 python bench.py --steps 2000 --warmup 100 --ref-client-requests 0" \
 "b_def2:200:python bench.py --steps 2000 --warmup 100 --ref-client-requests 0" \
 "b_wide2:300:TFSERVE_GRAPH_TUNE_TOP=12 TFSERVE_GRAPH_TUNE_RATIO=2.5 python bench.py --steps 2000 --warmup 100 --ref-client-requests 0" \
 "b1split:300:TFSERVE_SPLITK_FIXUP=1 python scripts/wg_trace.py --batch 1 --layers s2_3x3 s3_3x3 s3_1x1_in s4_3x3 s4_1x1_in --cfgs 51:1 51:2 51:4 36:1 36:2 36:4 54:1 54:4"
