set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
run() {  # name cfg splits
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE -d /tmp/pmc_$1 -o run -- python scripts/one_conv.py --h 7 --cin 512 --cout 512 --k 3 --s 1 --cfg $2 --splits $3 --iters 20 > /tmp/pmc_$1.log 2>&1 && python scripts/pmc_summary.py /tmp/pmc_$1 > gpurun_out/pmc_s4_$1.txt
}
run c36 36 1 && run c54 54 1 && run c32s4 32 4 && run c51 51 1
echo done
