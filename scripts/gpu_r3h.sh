#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3h
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d /tmp/prof_f -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 --graph-tune 0 > gpurun_out/r3h/pmc_f_run.log 2>&1 &&
python scripts/pmc_summary.py /tmp/prof_f --replay stem > gpurun_out/r3h/pmc_fetch_r50_b32.txt 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -d /tmp/prof_w -o run -- python scripts/bench_engine.py --model resnet50 --batch 32 --iters 3 --graph-tune 0 > gpurun_out/r3h/pmc_w_run.log 2>&1 &&
python scripts/pmc_summary.py /tmp/prof_w --replay stem > gpurun_out/r3h/pmc_write_r50_b32.txt 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --steps 200 --warmup 20 --ref-client-requests 12000 > gpurun_out/r3h/bench4_gloo.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 --ref-client-requests 12000 > gpurun_out/r3h/bench1.log 2>&1
rc=$?
rm -rf /tmp/prof_f /tmp/prof_w
exit $rc
