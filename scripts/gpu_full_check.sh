#!/bin/bash
# Round-end rehearsal on one GPU: the whole GPU suite, smoke(), then the 1-GPU bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full_gpusuite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 300 --warmup 30 > gpurun_out/full_bench.log 2>&1
