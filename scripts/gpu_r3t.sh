set -o pipefail
mkdir -p gpurun_out/r3t
export TMPDIR=/tmp
timeout -k 10 300 python scripts/probe_concurrency.py > gpurun_out/r3t/probe_oldtable.log 2>&1 &&
TFSERVE_TUNED_CACHE=0 timeout -k 10 600 python scripts/probe_concurrency.py --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3t/tuned_r50.json > gpurun_out/r3t/tune_r50.log 2>&1 &&
TFSERVE_TUNED_CACHE=0 timeout -k 10 600 python scripts/probe_concurrency.py --model bert-base --buckets 1 2 4 8 16 --save-tuned gpurun_out/r3t/tuned_bert.json > gpurun_out/r3t/tune_bert.log 2>&1 &&
TFSERVE_TUNED_CACHE=gpurun_out/r3t/tuned_r50.json timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3t/engine_newtable.log 2>&1 &&
timeout -k 10 300 python scripts/bench_engine.py --model resnet50 --batch 1 32 > gpurun_out/r3t/engine_oldtable.log 2>&1
