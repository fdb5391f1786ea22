#!/bin/bash
# flow kernel knob sweep at batch 1 / 4 (engine graph replay)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3x
run() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/bench_engine.py --model resnet50 --batch 1 4 > gpurun_out/r3x/$name.log 2>&1 || exit 1
  echo "$name $(grep -h '"batch": 1,' gpurun_out/r3x/$name.log | cut -c1-70) | $(grep -h '"batch": 4,' gpurun_out/r3x/$name.log | cut -c1-70)"
}
run base TFSERVE_FLOW=1
run split1 TFSERVE_FLOW_MAX_SPLITS=1
run split4 TFSERVE_FLOW_MAX_SPLITS=4
run spin TFSERVE_FLOW_DBG=4
run noacq TFSERVE_FLOW_DBG=1
run grid1 TFSERVE_FLOW_GRID_MULT=1
run target512 TFSERVE_FLOW_TARGET=512
run nowait TFSERVE_FLOW_DBG=2
