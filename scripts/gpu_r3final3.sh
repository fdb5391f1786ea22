#!/bin/bash
# HEAD check after the placement change: full GPU suite, smoke, the driver's 1-GPU command, a 300-step bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3final3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3final3/gpu_suite.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3final3/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3final3/driver20.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 300 --warmup 30 > gpurun_out/r3final3/bench300.log 2>&1
rc=$?
tail -3 gpurun_out/r3final3/gpu_suite.log
grep -h '^{' gpurun_out/r3final3/driver20.log gpurun_out/r3final3/bench300.log | cut -c1-200
exit $rc
