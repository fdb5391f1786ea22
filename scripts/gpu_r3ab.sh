#!/bin/bash
# BERT attention query-block sweep (TFSERVE_ATTN_QB) + kernel tests at QB=32/128
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ab
for qb in 32 128 64 32 128 64; do
  TFSERVE_ATTN_QB=$qb timeout -k 10 300 python -u scripts/bench_engine.py --model bert-base --batch 32 > gpurun_out/r3ab/engine_bert_qb$qb.log 2>&1 || exit 1
  echo "qb=$qb $(grep -h '"batch"' gpurun_out/r3ab/engine_bert_qb$qb.log | cut -c1-80)"
done
TFSERVE_ATTN_QB=32 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/r3ab/attn_qb32_tests.log 2>&1 &&
TFSERVE_ATTN_QB=128 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/r3ab/attn_qb128_tests.log 2>&1
