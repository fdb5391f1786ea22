#!/bin/bash
# flow kernel ablations (timing only): acquire fence, dependency waits
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3w
for d in 0 1 2 3; do
  TFSERVE_FLOW_DBG=$d timeout -k 10 200 python -u scripts/bench_engine.py --model resnet50 --batch 1 4 > gpurun_out/r3w/engine_dbg$d.log 2>&1 || exit 1
done
