#!/bin/bash
# One PMC pass over a model's HIP-graph replay; per-dispatch (per-layer) table
# -> gpurun_out/pmc_replay_<model>_b<batch>[_<tag>].txt
#   PASS=sq    (default) SQ / GRBM: MFMA busy, wait, active per layer
#   PASS=fetch FETCH_SIZE (3 TCC slots) + GRBM_GUI_ACTIVE: bytes read from beyond L2
#   PASS=write WRITE_SIZE (2 TCC slots) + GRBM_GUI_ACTIVE: bytes written
#   PASS=lds   LDS instructions, bank-conflict cycles, LDS wait per layer
# (FETCH_SIZE and WRITE_SIZE do not fit one pass: MI355X_MICROARCH.md PMC slots.)
# pmc_summary.py turns the byte counters into GB/s per layer and a bound class.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODEL=${MODEL:-resnet50}
BATCH=${BATCH:-32}
FIRST=${FIRST:-stem_pool}
PASS=${PASS:-sq}
case $PASS in
  sq) CTR="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"; TAG="";;
  fetch) CTR="FETCH_SIZE GRBM_GUI_ACTIVE"; TAG="_fetch";;
  write) CTR="WRITE_SIZE GRBM_GUI_ACTIVE"; TAG="_write";;
  lds) CTR="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; TAG="_lds";;
  *) echo "unknown PASS=$PASS"; exit 2;;
esac
rm -rf /tmp/prof_pmc
timeout -s KILL 280 rocprofv3 --pmc $CTR -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model $MODEL --batch $BATCH --iters 3 --graph-tune 0 > /tmp/pmc_run.log 2>&1 &&
python scripts/pmc_summary.py /tmp/prof_pmc --replay $FIRST > gpurun_out/pmc_replay_${MODEL}_b${BATCH}${TAG}.txt
rc=$?
tail -5 /tmp/pmc_run.log > gpurun_out/pmc_run_tail${TAG}.log
rm -rf /tmp/prof_pmc
exit $rc
