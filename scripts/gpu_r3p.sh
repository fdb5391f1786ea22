set -o pipefail
mkdir -p gpurun_out/r3p
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv_chain or halo_conv_is_det" > gpurun_out/r3p/tests_chain.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r3p/tests_resnet.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3p/engine.log 2>&1 &&
TFSERVE_CONV_CHAIN=0 timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3p/engine_nochain.log 2>&1 &&
timeout -k 10 300 python scripts/probe_concurrency.py > gpurun_out/r3p/probe.log 2>&1 &&
FIRST=stem_pool BATCH=32 bash scripts/gpu_trace_b1.sh
