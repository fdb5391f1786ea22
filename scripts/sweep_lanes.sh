#!/bin/bash
# 1-GPU sweep of bench.py lane count x in-flight RPCs (ResNet-50 b32, native transport).
# Each run is bounded by its own timeout; the first failing step ends the sweep.
set -e
mkdir -p gpurun_out/sweep_lanes
for lanes in 3 4 6; do
  for conc in 128 192 256; do
    timeout -k 10 120 python -u bench.py --lanes $lanes --concurrency $conc \
      > gpurun_out/sweep_lanes/l${lanes}_c${conc}.log 2>&1
    echo "lanes=$lanes conc=$conc $(tail -1 gpurun_out/sweep_lanes/l${lanes}_c${conc}.log | cut -c1-200)"
  done
done
