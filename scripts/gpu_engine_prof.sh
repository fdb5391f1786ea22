#!/bin/bash
# Engine timing + rocprofv3 kernel trace + one SQ/GRBM PMC pass of the ResNet-50
# b32 HIP-graph replay; summaries land in gpurun_out/*.txt, the raw databases
# are deleted on the box (gpurun copies back at most 64 MiB).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=${MODEL:-resnet50}
FIRST=${FIRST:-ingest}
scripts/gpu_session.sh \
 "engine:300:python scripts/bench_engine.py --model $MODEL --batch 1 32" \
 "kt:300:rocprofv3 --kernel-trace --stats -d /tmp/prof_kt -o run -- python scripts/bench_engine.py --model $MODEL --batch 32 --iters 20 && python scripts/replay_kernels.py \$(find /tmp/prof_kt -name '*.db' | head -1) --first $FIRST --list > gpurun_out/replay_${MODEL}.txt" \
 "pmc:300:timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model $MODEL --batch 32 --iters 3 --graph-tune 0 && python scripts/pmc_summary.py /tmp/prof_pmc > gpurun_out/pmc_${MODEL}.txt"
