#!/bin/bash
# usage: pmc_conv.sh TAG "one_conv.py args"  -> gpurun_out/pmc_conv_TAG.txt
# One PMC pass (LDS / MFMA / wait counters) over repeated launches of one conv config.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/pc_$1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d /tmp/pc_$1 -o run -- python scripts/one_conv.py $2 --iters 10 > /tmp/pc_$1.log 2>&1 && python scripts/pmc_summary.py /tmp/pc_$1 > gpurun_out/pmc_conv_$1.txt
