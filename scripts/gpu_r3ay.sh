#!/bin/bash
# multi-rank rehearsal on one GPU (gloo) with the L3 placement: self-launch 2 and 4 ranks, torchrun 2 ranks
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ay
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r3ay/self2.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r3ay/torchrun2.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 100 --warmup 10 > gpurun_out/r3ay/self4.log 2>&1
rc=$?
for f in self2 torchrun2 self4; do
  grep -h '^{' gpurun_out/r3ay/$f.log | python -c '
import sys, json
d = json.loads(sys.stdin.read())
print("'$f'", d["n_gpus"], d["value"], d["errors"], [x["placement"]["cpus"] for x in d["diagnostics"]])' || true
done
exit $rc
