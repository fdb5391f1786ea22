set -o pipefail
mkdir -p gpurun_out/r3j
export TMPDIR=/tmp
export TFSERVE_TUNED_CACHE=0
timeout -k 10 600 python scripts/probe_concurrency.py --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3j/tuned_r50.json > gpurun_out/r3j/tune_r50.log 2>&1 &&
timeout -k 10 600 python scripts/probe_concurrency.py --model bert-base --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3j/tuned_bert.json > gpurun_out/r3j/tune_bert.log 2>&1
