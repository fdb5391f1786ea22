set -o pipefail
mkdir -p gpurun_out/r3l
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py > gpurun_out/r3l/tests_resnet.log 2>&1 &&
bash scripts/gpu_r3j.sh &&
FIRST=stem_pool BATCH=1 bash scripts/gpu_trace_b1.sh &&
FIRST=embed MODEL=bert-base BATCH=32 bash scripts/gpu_trace_b1.sh
