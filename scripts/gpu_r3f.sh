set -o pipefail
mkdir -p gpurun_out/r3f
export TMPDIR=/tmp
TFSERVE_TUNED_CACHE=0 TFSERVE_GRAPH_TUNE_CONC=3 TFSERVE_GRAPH_TUNE_TOP=12 TFSERVE_GRAPH_TUNE_RATIO=10 TFSERVE_GRAPH_TUNE_MIN_US=0 timeout -k 10 900 python scripts/probe_concurrency.py --save-tuned gpurun_out/r3f/tuned_conc3_wide.json > gpurun_out/r3f/conc3_wide.log 2>&1
