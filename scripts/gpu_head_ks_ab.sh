#!/bin/bash
# A/B of the classifier head's K split (TFSERVE_HEAD_KS 4 vs 8) at b32: head
# tests, engine time and replay tables in each mode.
# usage: OUT=gpurun_out/<dir> bash scripts/gpu_head_ks_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="${OUT:-gpurun_out/head_ks}"
export OUT
mkdir -p "$OUT"
KT="cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace"
steps=(
  "heads:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k 'softmax or head or classifier'"
  "resnet:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py"
)
for ks in 4 8 4 8; do
  steps+=("eng_ks$ks:200:TFSERVE_HEAD_KS=$ks python -u scripts/bench_engine.py --batch 32")
done
for ks in 4 8; do
  steps+=("kt_ks$ks:200:export TFSERVE_HEAD_KS=$ks && $KT -d /tmp/kt$ks -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 && python scripts/replay_kernels.py \$(ls /tmp/kt$ks/*.db | tail -1) --first stem_pool --list > $OUT/replay_r50_b32_ks$ks.txt")
done
bash scripts/gpu_session.sh "${steps[@]}"
