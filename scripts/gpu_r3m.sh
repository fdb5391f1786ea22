set -o pipefail
mkdir -p gpurun_out/r3m
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_fastpath_gpu.py tests/test_kernels_gpu.py -k "not linear_matches and not conv_matches" > gpurun_out/r3m/tests.log 2>&1 &&
timeout -k 10 300 python scripts/probe_concurrency.py > gpurun_out/r3m/probe_r50.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r3m/bench1.log 2>&1 &&
TFSERVE_BF16_INGEST=0 timeout -k 10 400 python bench.py > gpurun_out/r3m/bench1_fp32ingest.log 2>&1
