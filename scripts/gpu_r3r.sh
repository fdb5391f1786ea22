set -o pipefail
mkdir -p gpurun_out/r3r
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "stem" tests/test_resnet_gpu.py > gpurun_out/r3r/tests_stem.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3r/engine.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 200 --warmup 20 --ref-client-requests 12000 > gpurun_out/r3r/bench2_gloo.log 2>&1 &&
timeout -k 10 500 python bench.py --model multi > gpurun_out/r3r/bench_multi.log 2>&1
