#!/bin/bash
# flow kernel: split / grid combinations at batch 1 / 2 / 4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3y
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/bench_engine.py --model resnet50 --batch 1 2 4 > gpurun_out/r3y/$name.log 2>&1 || exit 1
  echo "$name $(grep -h '"batch"' gpurun_out/r3y/$name.log | sed 's/.*"batch": \([0-9]*\), "graph_ms": \([0-9.]*\).*/b\1=\2/' | tr '\n' ' ')"
}
run split1_grid1 TFSERVE_FLOW_MAX_SPLITS=1 TFSERVE_FLOW_GRID_MULT=1
run split2_grid1 TFSERVE_FLOW_MAX_SPLITS=2 TFSERVE_FLOW_GRID_MULT=1
run split1_grid05 TFSERVE_FLOW_MAX_SPLITS=1 TFSERVE_FLOW_GRID_MULT=0.5
run split1_t128 TFSERVE_FLOW_MAX_SPLITS=2 TFSERVE_FLOW_TARGET=128 TFSERVE_FLOW_GRID_MULT=1
run noflow TFSERVE_FLOW=0
