set -o pipefail
mkdir -p gpurun_out/r3e
export TMPDIR=/tmp
TFSERVE_GRAPH_TUNE_CONC=1 timeout -k 10 300 python scripts/probe_concurrency.py > gpurun_out/r3e/conc_copies.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_bert_gpu.py tests/test_weights_gpu.py > gpurun_out/r3e/tests.log 2>&1 &&
timeout -k 10 600 python bench.py --model multi --reload-cycles 2 --bert-requests 3000 > gpurun_out/r3e/multi.log 2>&1
