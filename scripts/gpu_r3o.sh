set -o pipefail
mkdir -p gpurun_out/r3o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "conv_chain_is_det" > gpurun_out/r3o/det.log 2>&1
TFSERVE_CONV_CHAIN=0 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "share_one" > gpurun_out/r3o/pool_nochain.log 2>&1
TFSERVE_SHARED_GRAPH_POOL=0 timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_resnet_gpu.py -k "share_one" > gpurun_out/r3o/pool_private_chain.log 2>&1
echo done
