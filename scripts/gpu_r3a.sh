set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 120 python scripts/probe_topology.py torch > gpurun_out/r3a/probe.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/r3a/bench1.log 2>&1 &&
TFSERVE_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 200 --warmup 20 > gpurun_out/r3a/bench2_gloo.log 2>&1
