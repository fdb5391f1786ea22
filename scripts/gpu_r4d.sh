#!/bin/bash
# Round 4, session 4: tiny 2-rank rehearsal after the one-runner-per-tensor-set
# fix (rccl_ok), the reference-client phase with cache-hot (2) vs cold (64)
# bodies, the b32 (tail fusion on) and b1 replay kernel traces, one SQ PMC pass.
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
scripts/gpu_session.sh \
 "tiny2:300:TFSERVE_BENCH_BACKEND=gloo python bench.py --gpus 2 --model tiny --steps 2000 --warmup 100" \
 "bench_ref2:300:python bench.py --steps 2000 --warmup 100 --ref-client-requests 20000" \
 "bench_ref64:300:python bench.py --steps 2000 --warmup 100 --ref-client-requests 20000 --ref-client-bodies 64" \
 "kt32:300:TFSERVE_TAIL=1 rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 20 && python scripts/replay_kernels.py \$(find /tmp/prof_kt -name '*.db' | head -1) --first stem_pool --list > gpurun_out/replay_r50_b32_tail.txt" \
 "kt1:300:rm -rf /tmp/prof_kt1 && rocprofv3 --kernel-trace --stats -d /tmp/prof_kt1 -o run -- python scripts/bench_engine.py --model resnet50 --batch 1 --iters 20 && python scripts/replay_kernels.py \$(find /tmp/prof_kt1 -name '*.db' | head -1) --first stem_pool --list > gpurun_out/replay_r50_b1.txt" \
 "pmc:300:timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 --graph-tune 0 && python scripts/pmc_summary.py /tmp/prof_pmc --replay stem_pool > gpurun_out/pmc_r50_b32.txt"
