set -o pipefail
mkdir -p gpurun_out/r3k
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "linear_ln or strided or dense_softmax or linear_matches" > gpurun_out/r3k/tests_kernels.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bert_gpu.py > gpurun_out/r3k/tests_bert.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model bert-base --batch 1 32 > gpurun_out/r3k/bert_engine.log 2>&1 &&
TFSERVE_LN_FOLD=0 timeout -k 10 300 python scripts/bench_engine.py --model bert-base --batch 1 32 > gpurun_out/r3k/bert_engine_nofold.log 2>&1 &&
timeout -k 10 300 python scripts/prof_program_ops.py --model bert-base --batch 32 > gpurun_out/r3k/ops_bert.log 2>&1
