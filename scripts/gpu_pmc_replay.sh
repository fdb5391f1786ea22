#!/bin/bash
# One SQ/GRBM PMC pass over the ResNet-50 b32 HIP-graph replay; per-dispatch
# (per-layer) MFMA utilisation table -> gpurun_out/pmc_replay_<model>.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODEL=${MODEL:-resnet50}
BATCH=${BATCH:-32}
FIRST=${FIRST:-ingest}
timeout -s KILL 280 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model $MODEL --batch $BATCH --iters 3 --graph-tune 0 > /tmp/pmc_run.log 2>&1 &&
python scripts/pmc_summary.py /tmp/prof_pmc --replay $FIRST > gpurun_out/pmc_replay_${MODEL}_b${BATCH}.txt
rc=$?
tail -5 /tmp/pmc_run.log > gpurun_out/pmc_run_tail.log
rm -rf /tmp/prof_pmc
exit $rc
