#!/bin/bash
# PMC passes over the fused stem kernel (scripts/stem_bench.py), one counter group per run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=${BATCH:-32}
timeout -k 10 120 python scripts/stem_bench.py --batch $B > gpurun_out/stem_bench_b$B.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d /tmp/pmc_stem1 -o run -- python scripts/stem_bench.py --batch $B --iters 20 > /tmp/pmc_stem1.log 2>&1 &&
python scripts/pmc_summary.py /tmp/pmc_stem1 > gpurun_out/pmc_stem1_b$B.txt &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d /tmp/pmc_stem2 -o run -- python scripts/stem_bench.py --batch $B --iters 20 > /tmp/pmc_stem2.log 2>&1 &&
python scripts/pmc_summary.py /tmp/pmc_stem2 > gpurun_out/pmc_stem2_b$B.txt
