#!/bin/bash
# Round-6 closing session: head-kernel tests, the GPU suite, smoke, the
# driver command twice, engine timings and the b1 / b32 replay tables.
# usage: OUT=gpurun_out/<dir> bash scripts/gpu_final_r6.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT="${OUT:-gpurun_out/final}"
export OUT
mkdir -p "$OUT"
KT="cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace"
exec_steps=(
  "heads:200:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k 'softmax or head or classifier'"
  "suite:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
  "smoke:120:python -u -c 'import __graft_entry__ as g; g.smoke()'"
  "drv1:120:python -u bench.py --steps 20 --warmup 5"
  "drv2:120:python -u bench.py --steps 20 --warmup 5"
  "eng:200:python -u scripts/bench_engine.py --batch 1 32"
  "bert:200:python -u scripts/bench_engine.py --model bert-base --batch 32"
  "b1kt:200:$KT -d /tmp/ktr1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 && python scripts/replay_kernels.py \$(ls /tmp/ktr1/*.db | tail -1) --first h2d_rows --list > $OUT/replay_r50_b1.txt"
  "b32kt:200:$KT -d /tmp/ktr2 -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 && python scripts/replay_kernels.py \$(ls /tmp/ktr2/*.db | tail -1) --first stem_pool --list > $OUT/replay_r50_b32.txt"
)
bash scripts/gpu_session.sh "${exec_steps[@]}"
