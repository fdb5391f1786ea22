#!/bin/bash
# usage: pmc_gemm.sh TAG SHAPE CFG SPLITS
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pg_$1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d /tmp/pg_$1 -o run -- python scripts/gemm_one.py --shape $2 --cfg $3 --splits $4 --iters 10 > /tmp/pg_$1.log 2>&1 && python scripts/pmc_summary.py /tmp/pg_$1 > gpurun_out/pmc_gemm_$1.txt
