#!/bin/bash
# Round 4, session 7: BERT-base b32 engine with the PF cgemm candidates (+ its
# replay kernel table); headline A/B of the load generator's distinct request
# bodies (64 cold vs 4 cache-hot), interleaved on one box.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "bert:300:python scripts/bench_engine.py --model bert-base --batch 32" \
 "ab64a:200:python bench.py --steps 1000 --warmup 50 --ref-client-requests 0 --distinct-requests 64" \
 "ab4a:200:python bench.py --steps 1000 --warmup 50 --ref-client-requests 0 --distinct-requests 4" \
 "ab64b:200:python bench.py --steps 1000 --warmup 50 --ref-client-requests 0 --distinct-requests 64" \
 "ab4b:200:python bench.py --steps 1000 --warmup 50 --ref-client-requests 0 --distinct-requests 4" \
 "ktbert:300:rocprofv3 --kernel-trace --stats -d /tmp/prof_ktb -o run -- python scripts/bench_engine.py --model bert-base --batch 32 --iters 10 && python scripts/replay_kernels.py \$(find /tmp/prof_ktb -name '*.db' | head -1) --first embed_ln --list > gpurun_out/replay_bert_b32.txt"
