set -o pipefail
mkdir -p gpurun_out/r3b
export TMPDIR=/tmp
TFSERVE_GRAPH_TUNE_CONC=1 timeout -k 10 400 python scripts/probe_concurrency.py > gpurun_out/r3b/conc_iso.log 2>&1 &&
timeout -k 10 600 python scripts/probe_concurrency.py > gpurun_out/r3b/conc_tuned.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 300 --warmup 30 > gpurun_out/r3b/bench1.log 2>&1
