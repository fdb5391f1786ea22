#!/bin/bash
# Round 4, session 3: headline bench (busy-thread identities), the 2-rank gloo
# rehearsal (rccl block), the host ceiling probe (tiny model at 1 and 2 ranks on
# one box), the b32 replay kernel trace with the tail fusion on, and one SQ PMC
# pass (MFMA busy per layer).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "bench1:300:python bench.py --steps 2000 --warmup 100" \
 "gloo2:300:TFSERVE_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 1000 --warmup 50" \
 "tiny1:200:python bench.py --model tiny --steps 2000 --warmup 100" \
 "tiny2:300:TFSERVE_BENCH_BACKEND=gloo python bench.py --gpus 2 --model tiny --steps 2000 --warmup 100" \
 "kt_tail:300:TFSERVE_TAIL=1 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 && python scripts/replay_kernels.py \$(find /tmp/prof_kt -name '*.db' | head -1) --first ingest --list > gpurun_out/replay_r50_b32_tail.txt" \
 "pmc:300:timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 --graph-tune 0 && python scripts/pmc_summary.py /tmp/prof_pmc --replay ingest > gpurun_out/pmc_r50_b32.txt"
