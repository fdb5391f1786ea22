set -o pipefail
mkdir -p gpurun_out/r3s
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_resnet_gpu.py tests/test_bert_gpu.py tests/test_fastpath_gpu.py tests/test_multimodel_gpu.py tests/test_weights_gpu.py > gpurun_out/r3s/tests.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3s/engine.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model bert-base --batch 1 32 > gpurun_out/r3s/engine_bert.log 2>&1 &&
timeout -k 10 500 python bench.py --model multi > gpurun_out/r3s/bench_multi.log 2>&1 &&
timeout -k 10 400 python bench.py > gpurun_out/r3s/bench1.log 2>&1
