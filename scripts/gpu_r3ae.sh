#!/bin/bash
# multi-rank rehearsals on ONE GPU (gloo): the driver's torchrun launch (N=2) and the self-launch (N=4)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ae
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 10 > gpurun_out/r3ae/torchrun2.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 4 --steps 100 --warmup 10 > gpurun_out/r3ae/self4.log 2>&1
