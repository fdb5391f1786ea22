set -o pipefail
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "strided or dense_softmax or key_mask" tests/test_bert_gpu.py tests/test_weights_gpu.py > gpurun_out/r3d/tests.log 2>&1 &&
export TFSERVE_GRAPH_TUNE_CONC=1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 3 > gpurun_out/r3d/bench_l3.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 4 > gpurun_out/r3d/bench_l4_hwq8.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 4 --concurrency 192 > gpurun_out/r3d/bench_l4_c192.log 2>&1 &&
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 --lanes 6 --concurrency 192 > gpurun_out/r3d/bench_l6_hwq8_c192.log 2>&1
