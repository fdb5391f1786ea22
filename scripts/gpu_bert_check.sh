#!/bin/bash
# cgemm numerics (every config) + BERT tests + BERT-base b32 engine + one kernel-trace replay table.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-bert}
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_bert_gpu.py -k "cgemm or linear or splitk or attention or bert or layernorm or embedding" > gpurun_out/${TAG}_kernels.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_engine.py --model bert-base --batch 32 > gpurun_out/${TAG}_engine.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model bert-base --batch 32 --iters 20 > /tmp/kt.log 2>&1 &&
python scripts/replay_kernels.py $(find /tmp/prof_kt -name '*.db' | head -1) --first embed_ln --list > gpurun_out/${TAG}_replay_b32.txt
rc=$?
rm -rf /tmp/prof_kt
exit $rc
