#!/bin/bash
# Round-3 PMC passes over the ResNet-50 b32 HIP-graph replay (committed tile picks):
# pass 1 SQ/GRBM (MFMA busy, waits), pass 2 FETCH_SIZE, pass 3 WRITE_SIZE (one TCC group per pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3ah
pass() { # name, counters...
  local name=$1; shift
  rm -rf /tmp/prof_pmc
  timeout -s KILL 200 rocprofv3 --pmc "$@" -d /tmp/prof_pmc -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 > /tmp/pmc_run.log 2>&1 || { tail -5 /tmp/pmc_run.log > gpurun_out/r3ah/$name.err; return 1; }
  python scripts/pmc_summary.py /tmp/prof_pmc --replay stem_pool > gpurun_out/r3ah/pmc_$name.txt
}
pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE &&
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
pass write WRITE_SIZE GRBM_GUI_ACTIVE
rc=$?
rm -rf /tmp/prof_pmc
exit $rc
