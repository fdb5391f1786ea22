#!/bin/bash
# Back-to-back repeats of bench.py on one box: default config vs --lanes 6 --concurrency 256,
# interleaved so box drift hits both alike. Each run has its own timeout; first failure ends it.
set -e
mkdir -p gpurun_out/bench_repeat
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py > gpurun_out/bench_repeat/default_r${rep}.log 2>&1
  echo "default rep=$rep $(tail -1 gpurun_out/bench_repeat/default_r${rep}.log | cut -c1-170)"
  timeout -k 10 120 python -u bench.py --lanes 6 --concurrency 256 > gpurun_out/bench_repeat/l6c256_r${rep}.log 2>&1
  echo "l6c256 rep=$rep $(tail -1 gpurun_out/bench_repeat/l6c256_r${rep}.log | cut -c1-170)"
done
