set -o pipefail
mkdir -p gpurun_out/r3c
export TMPDIR=/tmp
export TFSERVE_GRAPH_TUNE_CONC=1
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python scripts/probe_concurrency.py --lanes 6 > gpurun_out/r3c/conc_hwq8_l6.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 3 > gpurun_out/r3c/bench_l3.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 4 > gpurun_out/r3c/bench_l4_hwq8.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 6 --concurrency 192 > gpurun_out/r3c/bench_l6_hwq8_c192.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 4 --concurrency 192 > gpurun_out/r3c/bench_l4_c192.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 4 > gpurun_out/r3c/bench_l4.log 2>&1
