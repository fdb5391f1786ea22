set -o pipefail
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --steps 200 --warmup 20 --ref-client-requests 12000 > gpurun_out/r3i/bench4_gloo.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 200 --warmup 20 --ref-client-requests 12000 > gpurun_out/r3i/bench2_gloo.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 TFSERVE_GRAPH_TUNE_CONC=1 timeout -k 10 300 python scripts/probe_concurrency.py --lanes 6 > gpurun_out/r3i/conc_hwq8_l6.log 2>&1
